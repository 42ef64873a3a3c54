// device_engine.hip — batched permission checks on MI355X (gfx950).
//
// Replaces the recursion of (*check.Engine).SubjectIsAllowed
// (internal/check/engine.go:33-95) for a whole batch of requests.  Without key
// collisions (R4) the reference answers "is the requested subject in the rows of the
// root query, or in the rows of some subject set reachable from them" (R2).  With
//   X(r)  = interior nodes reachable from root r through >= 1 edge,
//   rev(t) = expandable nodes whose rows contain subject t,
// that is:  allowed(r, t)  <=>  r in rev(t)  or  rev(t) ∩ X(r) != {}.
// The engine therefore
//   1. pushes a multi-source frontier over the INTERIOR subgraph only (subject-set
//      nodes that are themselves expandable), 64 requests per uint64 word, level by
//      level until no word gains a bit (no depth cutoff, R2), and
//   2. pulls once per request over rev(t) (a bottom-up step restricted to the
//      requested subject), testing the visited bit of its own word.
// Subject IDs (the bulk of all edges) are never traversed: they are only ever the last
// hop, which the pull resolves from the target side.
//
// Per-round HBM state (W words): vis[W][Ni] and nxt[W][Ni] (uint64), zero between
// rounds; every (word, node) that gets a bit is recorded in a frontier list or the
// `touch` list, and only those entries are reset (no O(N) clears).
//
// Kernels (one HIP stream per engine):
//   seed_kernel     one thread per request: level-0 frontier entries (word, root, bit)
//   expand_kernel   load-balanced push: 256-thread blocks take 1024-edge tiles of the
//                   level's concatenated rows, find their entries by a wave-cooperative
//                   search + an LDS binary search, OR masks into vis/nxt with 64-bit
//                   atomics and append new frontier entries with one packed atomic per
//                   wave (entry count in bits 36..63, row-length prefix in bits 0..35)
//   gather_kernel   next level's masks: nxt -> entry list, nxt cleared
//   pull_kernel     one thread per request, wave = one 64-request word (ballot)
//   reset_kernel    vis[...] = 0 for every recorded entry
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "core_index.hpp"
#include "device_util.hpp"
#include "labels.hpp"
#include "tier.hpp"
#include "ketogpu_internal.hpp"

using namespace ketogpu;
using namespace kdev;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;
constexpr uint32_t kDynBase = 0x80000000u;

struct DevGraph {
    const uint64_t *fint_off;
    const uint32_t *fint_col;
    const uint64_t *rev_off;
    const uint32_t *rev_col;
    const uint32_t *row_amb;  // nullptr when the snapshot has no ambiguous keys
    uint32_t Ni, Nx, N;
    uint32_t both_max, seed_max;  // bidi: both-sides and eager-seed thresholds (kBothMax, kSeedBothMax)
    // plan lite: added to every row begin an entry carries and taken off the record
    // arrays' base (0; a test knob, KETOGPU_TEST_BEGIN_SHIFT, that sends every begin
    // past 2^32 through the 64-bit path)
    uint64_t seed_shift;
    // plan core: node blocks of the seed rows per direction (core_index.hpp): node v's
    // block header is record blk[d] + (v << blk_log[d]) of that direction's array
    uint64_t blk[2];
    uint32_t blk_log[2];
    // hub index for the unit2 kernels (nullptr: off; see ketogpu_engine::build_hubs):
    // hub_of[v] (v < Nx) = hub number or NONE, hub_mask[v][hub_words] (v < Ni) bit h = v is
    // in the closure of hub h; forward edge records carry hub number + 1 in FRec::pad
    const uint32_t *hub_of;
    const uint64_t *hub_mask;
    uint32_t hub_words;
};

struct DevState {
    uint64_t *vis, *nxt;              // [W][Ni]
    uint64_t *fe_key, *fe_mask, *fe_pre;
    uint64_t fe_cap;
    uint64_t *touch;
    uint64_t touch_cap;
    unsigned long long *ctr;          // [0..1] level counters (ping-pong), [2] touch count
    unsigned int *overflow;
    unsigned long long *stats;        // [0] pull rev entries examined
    // hub index (nullptr: off): hub_of[v] (v < Nx) = hub number or NONE; hub_mask[v][k]
    // (v < Ni) bit j = v in closure+(hub 64k + j); hub_reach[request][k] bit j = the
    // request's search reached hub 64k + j (and did not expand it)
    const uint32_t *hub_of;
    const uint64_t *hub_mask;
    uint64_t *hub_reach;
    uint32_t hub_words;
};

// record that the requests in `bits` of word w reached hub h (its closure is in hub_mask)
__device__ __forceinline__ void hub_reached(const DevState &s, uint32_t w, uint64_t bits, uint32_t h) {
    for (uint64_t b = bits; b; b &= b - 1) {
        const uint64_t req = (uint64_t)w * 64 + (uint64_t)(__ffsll((unsigned long long)b) - 1);
        atomicOr((unsigned long long *)&s.hub_reach[req * s.hub_words + (h >> 6)], 1ull << (h & 63));
    }
}

__device__ __forceinline__ bool bit_of(const uint32_t *bm, uint32_t i) { return (bm[i >> 5] >> (i & 31)) & 1u; }

// Push mask m of word w into interior node u: returns the bits u gains.
__device__ __forceinline__ void push_one(const DevGraph &g, const DevState &s, uint32_t w, uint32_t u, uint64_t m,
                                         uint64_t *flags, uint32_t wglob, bool &app, uint64_t &deg, bool &touched) {
    size_t slot = (size_t)w * g.Ni + u;
    uint64_t cur = s.vis[slot];
    uint64_t nw = m & ~cur;
    if (!nw) return;
    uint64_t old = atomicOr((unsigned long long *)&s.vis[slot], (unsigned long long)nw);
    uint64_t newly = nw & ~old;
    if (!newly) return;
    if (g.row_amb && bit_of(g.row_amb, u)) atomicOr((unsigned long long *)&flags[wglob], (unsigned long long)newly);
    uint64_t d = g.fint_off[u + 1] - g.fint_off[u];
    if (s.hub_of) {  // a hub is visited but not expanded: its closure is looked up at the pull
        const uint32_t h = s.hub_of[u];
        if (h != KETOGPU_NODE_NONE) {
            hub_reached(s, w, newly, h);
            d = 0;
        }
    }
    if (d) {
        uint64_t o2 = atomicOr((unsigned long long *)&s.nxt[slot], (unsigned long long)newly);
        if (!o2) {
            app = true;
            deg = d;
        }
    } else if (!old) {
        touched = true;  // vis-only node: recorded once for the reset
    }
}

// ------------------------------------------------------------------- seed
__global__ __launch_bounds__(kBlock) void seed_kernel(DevGraph g, DevState s, const uint32_t *roots,
                                                      const uint32_t *targets, uint64_t c0, uint64_t n,
                                                      uint64_t *flags) {
    const int lane = threadIdx.x & 63;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;  // request index within the round
    bool want = false;
    uint64_t key = 0, deg = 0, mask = 0;
    if (i < n) {
        uint32_t r = roots[c0 + i], t = targets[c0 + i];
        if (r < g.Nx && t != KETOGPU_NODE_NONE) {
            uint64_t d = g.fint_off[r + 1] - g.fint_off[r];
            uint32_t w = (uint32_t)(i >> 6);
            mask = 1ull << (i & 63);
            if (g.row_amb && bit_of(g.row_amb, r)) atomicOr((unsigned long long *)&flags[(c0 + i) >> 6], mask);
            if (s.hub_of && d) {  // X(r) = closure+(r) for a hub root: nothing to expand
                const uint32_t h = s.hub_of[r];
                if (h != KETOGPU_NODE_NONE) {
                    hub_reached(s, w, mask, h);
                    d = 0;
                }
            }
            if (d) {
                want = true;
                key = ((uint64_t)w << 32) | r;
                deg = d;
            }
        }
    }
    wave_append(want, key, deg, lane, &s.ctr[0], 0, s.fe_cap, s.fe_key, s.fe_pre, s.fe_mask, mask, s.overflow);
}

// Dynamic roots (wildcard queries without a snapshot node): their interior rows come
// with the batch; push them directly into level 1 (rare path, one thread per request).
__global__ __launch_bounds__(kBlock) void seed_dynamic_kernel(DevGraph g, DevState s, const uint32_t *roots,
                                                              const uint32_t *targets, uint64_t c0, uint64_t n,
                                                              const uint64_t *dyn_int_off, const uint32_t *dyn_int,
                                                              const uint32_t *dyn_amb, uint64_t *flags,
                                                              uint64_t base1, unsigned long long *ctr1) {
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint32_t r = roots[c0 + i], t = targets[c0 + i];
    if (r < kDynBase || r == KETOGPU_NODE_NONE || t == KETOGPU_NODE_NONE) return;
    uint32_t k = r - kDynBase, w = (uint32_t)(i >> 6);
    uint64_t m = 1ull << (i & 63);
    uint32_t wglob = (uint32_t)((c0 + i) >> 6);
    if (dyn_amb[k]) atomicOr((unsigned long long *)&flags[wglob], m);
    for (uint64_t e = dyn_int_off[k]; e < dyn_int_off[k + 1]; e++) {
        uint32_t u = dyn_int[e];
        bool app = false, touched = false;
        uint64_t deg = 0;
        push_one(g, s, w, u, m, flags, wglob, app, deg, touched);
        uint64_t key = ((uint64_t)w << 32) | u;
        if (app) {
            uint64_t pos = atomicAdd(ctr1, (unsigned long long)((1ull << kCntShift) | deg));
            uint64_t idx = base1 + (pos >> kCntShift);
            if ((pos & kPreMask) + deg > kPreMask) atomicOr(s.overflow, 1u);  // prefix carry
            if (idx < s.fe_cap) {
                s.fe_key[idx] = key;
                s.fe_pre[idx] = pos & kPreMask;
            } else {
                atomicOr(s.overflow, 1u);
            }
        }
        if (touched) {
            uint64_t idx = atomicAdd(&s.ctr[2], 1ull);
            if (idx < s.touch_cap)
                s.touch[idx] = key;
            else
                atomicOr(s.overflow, 1u);
        }
    }
}

// ----------------------------------------------------------------- expand
__global__ __launch_bounds__(kBlock) void expand_kernel(DevGraph g, DevState s, uint64_t ent_begin, uint64_t ent_count,
                                                        uint64_t total_edges, uint64_t out_base,
                                                        unsigned long long *out_ctr, uint64_t *flags, uint64_t wg0) {
    __shared__ uint64_t s_pre[kTile + 1];
    __shared__ uint64_t s_first, s_count;
    const int lane = threadIdx.x & 63;
    const uint64_t *pre = s.fe_pre + ent_begin;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kTile; t0 < total_edges; t0 += (uint64_t)gridDim.x * kTile) {
        uint64_t t1 = t0 + kTile < total_edges ? t0 + kTile : total_edges;
        if (threadIdx.x < 64) {
            uint64_t i0 = wave_upper_bound(pre, ent_count, t0, lane) - 1;
            uint64_t i1 = wave_upper_bound(pre, ent_count, t1 - 1, lane) - 1;
            if (lane == 0) {
                s_first = i0;
                s_count = i1 - i0 + 1;
            }
        }
        __syncthreads();
        const uint64_t first = s_first, count = s_count;
        for (uint64_t j = threadIdx.x; j <= count; j += kBlock)
            s_pre[j] = (first + j < ent_count) ? pre[first + j] : total_edges;
        __syncthreads();
#pragma unroll 1
        for (int it = 0; it < kItems; it++) {
            uint64_t e = t0 + (uint64_t)it * kBlock + threadIdx.x;
            bool app = false, touched = false;
            uint64_t deg = 0, key = 0;
            if (e < t1) {
                // entry j: s_pre[j] <= e < s_pre[j+1]
                uint64_t lo = 0, hi = count;
                while (hi - lo > 1) {
                    uint64_t mid = (lo + hi) >> 1;
                    if (s_pre[mid] <= e)
                        lo = mid;
                    else
                        hi = mid;
                }
                uint64_t ent = ent_begin + first + lo;
                uint64_t k = s.fe_key[ent];
                uint32_t w = (uint32_t)(k >> 32), v = (uint32_t)k;
                uint64_t m = s.fe_mask[ent];
                uint32_t u = g.fint_col[g.fint_off[v] + (e - s_pre[lo])];
                push_one(g, s, w, u, m, flags, (uint32_t)(wg0 + w), app, deg, touched);
                key = ((uint64_t)w << 32) | u;
            }
            wave_append(app, key, deg, lane, out_ctr, out_base, s.fe_cap, s.fe_key, s.fe_pre, nullptr, 0,
                        s.overflow);
            wave_touch(touched, key, lane, &s.ctr[2], s.touch, s.touch_cap, s.overflow);
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------- gather
__global__ __launch_bounds__(kBlock) void gather_kernel(DevGraph g, DevState s, uint64_t b, uint64_t e) {
    uint64_t i = b + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= e) return;
    uint64_t k = s.fe_key[i];
    size_t slot = (size_t)(k >> 32) * g.Ni + (uint32_t)k;
    s.fe_mask[i] = s.nxt[slot];
    s.nxt[slot] = 0;
}

// ------------------------------------------------------------------- pull
__global__ __launch_bounds__(kBlock) void pull_kernel(DevGraph g, DevState s, const uint32_t *roots, const uint32_t *targets,
                                                      uint64_t c0, uint64_t n, const uint64_t *dyn_full_off,
                                                      const uint32_t *dyn_full, uint64_t *allowed) {
    const int lane = threadIdx.x & 63;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool ok = false;
    uint64_t examined = 0;
    if (i < n) {
        uint32_t r = roots[c0 + i], t = targets[c0 + i];
        if (r != KETOGPU_NODE_NONE && t != KETOGPU_NODE_NONE) {
            const uint64_t *vrow = s.vis + (size_t)(i >> 6) * g.Ni;
            const int b = (int)(i & 63);
            if (r >= kDynBase) {  // t in the dynamic root's rows?
                uint32_t k = r - kDynBase;
                uint64_t lo = dyn_full_off[k], hi = dyn_full_off[k + 1];
                while (lo < hi) {
                    uint64_t mid = (lo + hi) >> 1;
                    if (dyn_full[mid] < t)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                ok = lo < dyn_full_off[k + 1] && dyn_full[lo] == t;
            }
            const uint64_t pb = g.rev_off[t], pe = g.rev_off[t + 1];
            for (uint64_t p = pb; p < pe && !ok; p++) {
                uint32_t v = g.rev_col[p];
                examined++;
                if (v == r || (v < g.Ni && ((vrow[v] >> b) & 1ull))) ok = true;
            }
            // hubs this request reached: v is in X(r) if some reached hub's closure holds it.
            // Only the non-zero words of the request's reach bitmap are compared.
            const uint64_t *reach = s.hub_reach ? s.hub_reach + i * s.hub_words : nullptr;
            for (uint32_t k = 0; reach && k < s.hub_words && !ok; k++) {
                const uint64_t rk = reach[k];
                if (!rk) continue;
                for (uint64_t p = pb; p < pe && !ok; p++) {
                    uint32_t v = g.rev_col[p];
                    if (v >= g.Ni) break;  // rows are sorted: interior predecessors first
                    ok = (s.hub_mask[(size_t)v * s.hub_words + k] & rk) != 0;
                }
            }
        }
    }
    uint64_t bal = __ballot(ok);
    if (lane == 0 && i < n) allowed[(c0 + i) >> 6] = bal;
    // one atomic per wave for the statistics
    for (int d = 32; d; d >>= 1) examined += __shfl_down(examined, d, 64);
    if (lane == 0 && examined) atomicAdd(&s.stats[0], (unsigned long long)examined);
}

// ------------------------------------------------------------------ reset
__global__ __launch_bounds__(kBlock) void reset_kernel(uint64_t *vis, uint32_t Ni, const uint64_t *keys, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    uint64_t k = keys[i];
    vis[(size_t)(k >> 32) * Ni + (uint32_t)k] = 0;
}

// hub index build: the closures of the round's requests (hubs w0*64 ...) into hub_mask
__global__ __launch_bounds__(kBlock) void hub_mask_kernel(const uint64_t *vis, uint32_t Ni, uint64_t nw, uint32_t w0,
                                                          uint32_t hub_words, uint64_t *hub_mask) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nw * Ni; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t w = i / Ni, v = i - w * Ni;
        hub_mask[v * hub_words + w0 + w] = vis[i];
    }
}

// ------------------------------------------------------- LDS unit traversal
// The fast path.  One 256-thread workgroup takes a UNIT of U consecutive requests and
// runs the whole check for them — seed, every BFS level over the interior subgraph,
// and the rev(t) pull — with the unit's visited and pending bits in an LDS hash table
// (node -> U visited bits | U pending bits).  HBM only serves read-only graph rows: no
// global atomics, no state to reset, no host round trip per level.  Units whose
// closure outgrows the table (or that have a dynamic root) SPILL: 16-request units are
// re-run as 4-request units, those as single requests, and only single requests whose
// closure exceeds the table go to the global multi-word engine.
// unit_kernel / unit2_kernel LDS table: 2^KETO_U2_HASHLOG slots (build knob for A/B)
#ifndef KETO_U2_HASHLOG
#define KETO_U2_HASHLOG 11
#endif
constexpr int kHashLog = KETO_U2_HASHLOG;
constexpr int kHash = 1 << kHashLog;
constexpr int kHashMax = kHash * 3 / 4;
constexpr int kChunk = kBlock;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kUnitMax = 16;

struct UnitShared {
    uint32_t key[kHash];
    uint32_t st[kHash];  // visited bits (low 16) | pending bits (high 16)
    uint16_t cur_slot[kHash], cur_mask[kHash], nxt_slot[kHash];
    uint64_t c_begin[kChunk];
    uint32_t c_pre[kChunk + 1];
    uint16_t c_mask[kChunk];
    uint32_t wave_sum[kBlock / 64];
    uint32_t root[kUnitMax], target[kUnitMax];
    uint32_t n_used, n_nxt, spill, res;
    unsigned long long cnt_rows, cnt_edges, cnt_rev;
};

__device__ __forceinline__ uint32_t hslot(uint32_t u) { return (u * 2654435761u) >> (32 - kHashLog); }

__device__ __forceinline__ uint32_t lanes_below(uint64_t bal) {
    return (uint32_t)__popcll(bal & ((1ull << (threadIdx.x & 63)) - 1));
}

// exclusive block scan of one u32 per thread; returns the total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *out_pre, UnitShared &S) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    if (lane == 63) S.wave_sum[wv] = x;
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; i++) {
        uint32_t s = S.wave_sum[i];
        base += i < wv ? s : 0;
        total += s;
    }
    out_pre[tid] = base + x - v;
    if (tid == 0) out_pre[kBlock] = total;
    __syncthreads();
    return total;
}

// Insert u with mask m (want = this lane has an edge).  Called by whole waves: the
// occupancy counter and the next-frontier list are advanced with one LDS atomic per wave.
__device__ __forceinline__ void unit_push(const DevGraph &g, UnitShared &S, bool want, uint32_t u, uint32_t m,
                                          const uint32_t *has_kids, uint64_t *flag_word, int shift) {
    int h = -1;
    bool inserted = false;
    if (want) {
        uint32_t hh = hslot(u);
        for (int p = 0; p < kHash; p++, hh = (hh + 1) & (kHash - 1)) {
            uint32_t kv = S.key[hh];
            if (kv == kEmpty) {
                uint32_t prev = atomicCAS(&S.key[hh], kEmpty, u);
                if (prev == kEmpty) {
                    inserted = true;
                    h = (int)hh;
                    break;
                }
                kv = prev;
            }
            if (kv == u) {
                h = (int)hh;
                break;
            }
        }
        if (h < 0) S.spill = 1;  // table full
    }
    uint64_t bal = __ballot(inserted);
    if (bal && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)bal) - 1))
        if (atomicAdd(&S.n_used, (uint32_t)__popcll(bal)) + (uint32_t)__popcll(bal) > (uint32_t)kHashMax) S.spill = 1;
    bool app = false;
    if (h >= 0) {
        uint32_t old = atomicOr(&S.st[h], m);
        uint32_t newly = m & ~old & 0xFFFFu;
        if (newly) {
            if (g.row_amb && bit_of(g.row_amb, u))
                atomicOr((unsigned long long *)flag_word, (unsigned long long)newly << shift);
            if (bit_of(has_kids, u)) {
                uint32_t o2 = atomicOr(&S.st[h], newly << 16);
                app = !(o2 >> 16);
            }
        }
    }
    uint64_t ab = __ballot(app);
    if (ab) {
        int leader = __ffsll((unsigned long long)ab) - 1;
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&S.n_nxt, (uint32_t)__popcll(ab));
        base = __shfl(base, leader, 64);
        if (app) S.nxt_slot[base + lanes_below(ab)] = (uint16_t)h;
    }
}

__device__ __forceinline__ int unit_lookup(const UnitShared &S, uint32_t v) {
    uint32_t h = hslot(v);
    for (int p = 0; p < kHash; p++, h = (h + 1) & (kHash - 1)) {
        uint32_t kv = S.key[h];
        if (kv == v) return (int)h;
        if (kv == kEmpty) return -1;
    }
    return -1;
}

// Unit statistics are summed into kStatSlots spread slots (4 u64 each, from stats[8]):
// tens of thousands of workgroups adding to ONE address serialize at the memory side
// (~12 ns per atomic) and that alone cost ~2 ms per 1M requests.
constexpr int kStatSlots = 1024;
// statistics buffer: [8 misc][2 regions x 4 * kStatSlots][8 reduced][spill counters]
constexpr int kStatsLen = 8 + 8 * kStatSlots + 8 + 4;
__device__ __forceinline__ unsigned long long *stat_slot(unsigned long long *stats) {
    return stats + 8 + (size_t)(blockIdx.x & (kStatSlots - 1)) * 4;
}

// per-wave reduction of three counters, then one LDS atomic each per wave (all 256
// threads hitting one address serializes ~768 atomics per unit)
__device__ __forceinline__ void wave_stats_add(uint64_t a, uint64_t b, uint64_t c, unsigned long long *pa,
                                               unsigned long long *pb, unsigned long long *pc) {
#pragma unroll
    for (int s = 32; s; s >>= 1) {
        a += __shfl_down(a, s, 64);
        b += __shfl_down(b, s, 64);
        c += __shfl_down(c, s, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(pa, (unsigned long long)a);
        atomicAdd(pb, (unsigned long long)b);
        atomicAdd(pc, (unsigned long long)c);
    }
}

// expand the chunk held in S.c_begin / S.c_pre / S.c_mask (entries [0, k)); the loop
// count is block-uniform so every wave reaches the aggregated atomics together
__device__ __forceinline__ void unit_expand_chunk(const DevGraph &g, UnitShared &S, uint32_t k, uint32_t total,
                                                  const uint32_t *has_kids, uint64_t *flag_word, int shift,
                                                  uint64_t &edges) {
    for (uint32_t base = 0; base < total; base += kBlock) {
        uint32_t e = base + threadIdx.x;
        bool want = e < total;
        uint32_t u = 0, m = 0;
        if (want) {
            uint32_t lo = 0, hi = k;  // largest j with c_pre[j] <= e
            while (hi - lo > 1) {
                uint32_t mid = (lo + hi) >> 1;
                if (S.c_pre[mid] <= e)
                    lo = mid;
                else
                    hi = mid;
            }
            u = g.fint_col[S.c_begin[lo] + (e - S.c_pre[lo])];
            m = S.c_mask[lo];
            edges++;
        }
        unit_push(g, S, want, u, m, has_kids, flag_word, shift);
    }
}

// U requests per unit.  Pass 1 (parents == nullptr): unit b = requests [U*b, U*b+U).
// Later passes split the spilled units of the previous pass (size U*fan) into `fan`
// units each: unit b = child fan*parents[b/fan] + b%fan.  Spilled units are appended to
// spill_out (in units of U).
template <int U>
__global__ __launch_bounds__(kBlock) void unit_kernel(DevGraph g, const uint32_t *has_kids, const uint32_t *roots,
                                                      const uint32_t *targets, uint64_t n, uint64_t *allowed,
                                                      uint64_t *flags, const uint32_t *parents, uint32_t fan,
                                                      uint32_t *spill_out, unsigned int *spill_count,
                                                      unsigned long long *stats, unsigned long long *stamps) {
    __shared__ UnitShared S;
    const int tid = threadIdx.x;
    // diagnostic build only (stamps != nullptr): s_memtime at phase boundaries
    unsigned long long *stamp = (stamps && blockIdx.x < 65536 && tid == 0) ? stamps + (size_t)blockIdx.x * 16 : nullptr;
    uint32_t n_levels = 0;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();
    const uint64_t unit = parents ? (uint64_t)parents[blockIdx.x / fan] * fan + blockIdx.x % fan : blockIdx.x;
    const uint64_t c0 = unit * U;
    uint64_t *flag_word = &flags[c0 >> 6];
    const int shift = (int)(c0 & 63);
    const unsigned long long unit_bits = (U == 64 ? ~0ull : ((1ull << U) - 1)) << shift;
    for (int i = tid; i < kHash; i += kBlock) {
        S.key[i] = kEmpty;
        S.st[i] = 0;
    }
    if (tid == 0) {
        S.n_used = S.n_nxt = S.spill = S.res = 0;
        S.cnt_rows = S.cnt_edges = S.cnt_rev = 0;
    }
    if (tid < U) {
        uint64_t c = c0 + tid;
        uint32_t r = KETOGPU_NODE_NONE, t = KETOGPU_NODE_NONE;
        if (c < n) {
            r = roots[c];
            t = targets[c];
        }
        if (t == KETOGPU_NODE_NONE) r = KETOGPU_NODE_NONE;  // nothing can match
        S.root[tid] = r;
        S.target[tid] = t;
    }
    __syncthreads();
    if (tid < U && S.root[tid] != KETOGPU_NODE_NONE && S.root[tid] >= kDynBase) S.spill = 1;
    __syncthreads();
    if (S.spill) {
        if (tid == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        return;
    }
    uint64_t rows = 0, edges = 0, rev = 0;
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();
    // level 0: the roots' interior successors (roots themselves are not visited)
    {
        uint32_t d = 0;
        if (tid < U) {
            uint32_t r = S.root[tid];
            uint64_t b = 0;
            if (r != KETOGPU_NODE_NONE) {
                b = g.fint_off[r];
                d = (uint32_t)(g.fint_off[r + 1] - b);
                rows++;
                if (g.row_amb && bit_of(g.row_amb, r))
                    atomicOr((unsigned long long *)flag_word, (unsigned long long)1 << (shift + tid));
            }
            S.c_begin[tid] = b;
            S.c_mask[tid] = (uint16_t)(1u << tid);
        }
        uint32_t total = block_excl_scan(d, S.c_pre, S);
        unit_expand_chunk(g, S, U, total, has_kids, flag_word, shift, edges);
    }
    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();
    // levels until no request of the unit gains a bit (no depth cutoff)
    for (;;) {
        __syncthreads();
        uint32_t cnt = S.n_nxt;
        if (S.spill || !cnt) break;
        n_levels++;
        for (uint32_t i = tid; i < cnt; i += kBlock) {
            uint16_t s = S.nxt_slot[i];
            S.cur_slot[i] = s;
            S.cur_mask[i] = (uint16_t)(atomicAnd(&S.st[s], 0xFFFFu) >> 16);
        }
        __syncthreads();
        if (tid == 0) S.n_nxt = 0;
        for (uint32_t base = 0; base < cnt; base += kChunk) {
            uint32_t k = cnt - base < (uint32_t)kChunk ? cnt - base : (uint32_t)kChunk;
            uint32_t d = 0;
            if ((uint32_t)tid < k) {
                uint32_t v = S.key[S.cur_slot[base + tid]];
                uint64_t b = g.fint_off[v];
                d = (uint32_t)(g.fint_off[v + 1] - b);
                S.c_begin[tid] = b;
                S.c_mask[tid] = S.cur_mask[base + tid];
                rows++;
            }
            uint32_t total = block_excl_scan(d, S.c_pre, S);
            unit_expand_chunk(g, S, k, total, has_kids, flag_word, shift, edges);
            __syncthreads();
        }
    }
    if (S.spill) {
        if (tid == 0) {
            spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
            atomicAnd((unsigned long long *)flag_word, ~unit_bits);
        }
        return;
    }
    if (stamp) stamp[3] = __builtin_amdgcn_s_memtime();
    // pull: kBlock / U lanes per request over rev(target)
    {
        constexpr int L = kBlock / U;
        const int j = tid / L, l = tid % L;
        bool ok = false;
        uint32_t r = S.root[j], t = S.target[j];
        if (r != KETOGPU_NODE_NONE) {
            uint64_t b = g.rev_off[t], e = g.rev_off[t + 1];
            if (l == 0) rows++;
            for (uint64_t p = b + l; p < e && !ok; p += L) {
                uint32_t v = g.rev_col[p];
                rev++;
                if (v == r) {
                    ok = true;
                } else if (v < g.Ni) {
                    int s = unit_lookup(S, v);
                    ok = s >= 0 && ((S.st[s] >> j) & 1u);
                }
            }
        }
        if (ok) atomicOr(&S.res, 1u << j);
    }
    wave_stats_add(rows, edges, rev, &S.cnt_rows, &S.cnt_edges, &S.cnt_rev);
    __syncthreads();
    if (stamp) {
        stamp[4] = __builtin_amdgcn_s_memtime();
        stamp[5] = n_levels;
        stamp[6] = S.n_used;
        stamp[7] = 1;  // completed (not spilled)
    }
    if (tid == 0) {
        if (S.res) atomicOr((unsigned long long *)&allowed[c0 >> 6], (unsigned long long)S.res << shift);
        atomicAdd(&stat_slot(stats)[0], S.cnt_rows);
        atomicAdd(&stat_slot(stats)[1], S.cnt_edges);
        atomicAdd(&stat_slot(stats)[2], S.cnt_rev);
    }
}

// ------------------------------------------------------ unit traversal v2
// Measured (s_memtime stamps, config #2): a unit lived ~60k cycles, 24k of them in the
// pull (rev_off -> rev_col, two dependent HBM misses) and ~11k per BFS level (row
// offsets -> row entries, two dependent loads + scan/barriers).  v2 removes one
// dependent load per level and hides the pull's:
//   * edge RECORDS {node, interior degree, row begin}: pushing a node yields the row
//     of the next level, so a level costs one dependent global load (the records);
//   * each request's reverse row is prefetched into LDS (first kRevCache entries) while
//     the BFS runs; the pull is then LDS-only for targets with <= kRevCache entries.
struct FRec {
    uint32_t node, deg, begin, pad;
};

// Writable snapshots: rewrite patched rows in place (engine::sync).  seg holds
// (destination, source, length, 0 = forward row / 1 = reverse row) per row; one workgroup
// per row (grid-stride), the records only where the engine keeps them.
__global__ __launch_bounds__(256) void patch_rows_kernel(const uint64_t *seg, uint64_t nseg, const uint32_t *cols,
                                                         const FRec *recs, uint32_t *fint_col, FRec *frec,
                                                         uint32_t *rev_col, FRec *brec) {
    for (uint64_t i = blockIdx.x; i < nseg; i += gridDim.x) {
        const uint64_t dst = seg[4 * i], src = seg[4 * i + 1], len = seg[4 * i + 2];
        const bool rev = seg[4 * i + 3] != 0;
        uint32_t *col = rev ? rev_col : fint_col;
        FRec *rec = rev ? brec : frec;
        for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) {
            col[dst + k] = cols[src + k];
            if (rec) rec[dst + k] = recs[src + k];
        }
    }
}
// unit2 frontier entries per level (spill beyond).  256 (round 2; 512 before): 25.6 instead
// of 31 KB of LDS per unit, 6 instead of 5 units per CU for this latency-bound kernel —
// config #3 at 500M tuples 6.5 -> 7.7 x 10^8 checks/s, 0 spills (Kernels)
#ifndef KETO_U2_FRONT
#define KETO_U2_FRONT 256
#endif
constexpr int kFront = KETO_U2_FRONT;
constexpr int kRevCache = 16;
constexpr int kHubList = 128;  // hubs a unit may reach (spill beyond)

// Table shape per unit size: 16- and 4-request units keep 2^kHashLog slots and kFront
// frontier entries; the single-request stage (the last before the multi-word global path)
// takes most of a CU's LDS — 2^14 slots, 512 entries per level, ~142 KB, one workgroup per
// CU — so a closure of up to 12k non-hub nodes stays in LDS (round 3: with 2048 slots, 304
// of 10^6 config #4-shape requests at 200M tuples went on to the host-driven global path,
// ~0.8 ms of a 1.6 ms step).
#ifndef KETO_U2_HLOG1
#define KETO_U2_HLOG1 14
#endif
#ifndef KETO_U2_FRONT1
#define KETO_U2_FRONT1 512
#endif
#ifndef KETO_U2_HUBS1
#define KETO_U2_HUBS1 1024
#endif
#ifndef KETO_U2_HUBS
#define KETO_U2_HUBS kHubList
#endif
template <int U>
struct Unit2Shape {
    static constexpr int HLOG = U == 1 ? KETO_U2_HLOG1 : kHashLog;
    static constexpr int H = 1 << HLOG;
    static constexpr int HMAX = H * 3 / 4;
    static constexpr int FRONT = U == 1 ? KETO_U2_FRONT1 : kFront;
    static constexpr int HUBS = U == 1 ? KETO_U2_HUBS1 : KETO_U2_HUBS;  // hubs a unit may reach (spill beyond)
    static_assert(H <= 65535, "slots are kept in 16 bits (0xFFFF marks a hub root)");
};

template <int HLOG>
__device__ __forceinline__ uint32_t hslot_l(uint32_t u) {
    return (u * 2654435761u) >> (32 - HLOG);
}

template <int HLOG>
__device__ __forceinline__ int key_lookup_l(const uint32_t *key, uint32_t v) {
    constexpr int H = 1 << HLOG;
    uint32_t h = hslot_l<HLOG>(v);
    for (int p = 0; p < H; p++, h = (h + 1) & (H - 1)) {
        uint32_t kv = key[h];
        if (kv == v) return (int)h;
        if (kv == kEmpty) return -1;
    }
    return -1;
}

template <int U>
struct Unit2Shared {
    using Shape = Unit2Shape<U>;
    uint32_t key[Shape::H];
    uint32_t st[Shape::H];  // visited bits (low 16) | pending bits (high 16)
    uint16_t cur_slot[Shape::FRONT], cur_mask[Shape::FRONT], nxt_slot[Shape::FRONT];
    uint32_t cur_begin[Shape::FRONT], cur_deg[Shape::FRONT], nxt_begin[Shape::FRONT], nxt_deg[Shape::FRONT];
    uint32_t c_pre[kChunk + 1];
    uint32_t wave_sum[kBlock / 64];
    uint32_t root[U], target[U], rev_n[U];
    uint64_t rev_b[U];
    uint32_t rev_c[U][kRevCache];
    // hubs reached (hub index on): hub number, table slot (its visited bits are the
    // requests that reached it) or 0xFFFF for a hub ROOT, whose requests are hub_bits
    uint32_t hub_id[Shape::HUBS];
    uint16_t hub_slot[Shape::HUBS], hub_bits[Shape::HUBS];
    uint32_t n_used, n_nxt, spill, res, n_hub;
    unsigned long long cnt_rows, cnt_edges, cnt_rev;
};

template <int U>
__device__ __forceinline__ uint32_t block_excl_scan2(uint32_t v, Unit2Shared<U> &S) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    if (lane == 63) S.wave_sum[wv] = x;
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; i++) {
        uint32_t s = S.wave_sum[i];
        base += i < wv ? s : 0;
        total += s;
    }
    S.c_pre[tid] = base + x - v;
    if (tid == 0) S.c_pre[kBlock] = total;
    __syncthreads();
    return total;
}

template <int U>
__device__ __forceinline__ void unit2_push(const DevGraph &g, Unit2Shared<U> &S, bool want, const FRec &rc, uint32_t m,
                                           uint64_t *flag_word, int shift) {
    const uint32_t u = rc.node;
    int h = -1;
    bool inserted = false;
    if (want) {
        using Shape = Unit2Shape<U>;
        uint32_t hh = hslot_l<Shape::HLOG>(u);
        for (int p = 0; p < Shape::H; p++, hh = (hh + 1) & (Shape::H - 1)) {
            uint32_t kv = S.key[hh];
            if (kv == kEmpty) {
                uint32_t prev = atomicCAS(&S.key[hh], kEmpty, u);
                if (prev == kEmpty) {
                    inserted = true;
                    h = (int)hh;
                    break;
                }
                kv = prev;
            }
            if (kv == u) {
                h = (int)hh;
                break;
            }
        }
        if (h < 0) S.spill = 1;
    }
    const int lane = threadIdx.x & 63;
    uint64_t bal = __ballot(inserted);
    if (bal && lane == __ffsll((unsigned long long)bal) - 1) {
        uint32_t c = (uint32_t)__popcll(bal);
        if (atomicAdd(&S.n_used, c) + c > (uint32_t)Unit2Shape<U>::HMAX) S.spill = 1;
    }
    bool app = false;
    // a hub is visited but not expanded: the pull reads its closure from hub_mask
    const bool hub = g.hub_mask && rc.pad;
    if (inserted && hub) {
        uint32_t j = atomicAdd(&S.n_hub, 1u);
        if (j < (uint32_t)Unit2Shape<U>::HUBS) {
            S.hub_id[j] = rc.pad - 1;
            S.hub_slot[j] = (uint16_t)h;
        } else {
            S.spill = 1;
        }
    }
    if (h >= 0) {
        uint32_t old = atomicOr(&S.st[h], m);
        uint32_t newly = m & ~old & 0xFFFFu;
        if (newly) {
            if (g.row_amb && bit_of(g.row_amb, u))
                atomicOr((unsigned long long *)flag_word, (unsigned long long)newly << shift);
            if (rc.deg && !hub) {
                uint32_t o2 = atomicOr(&S.st[h], newly << 16);
                app = !(o2 >> 16);
            }
        }
    }
    uint64_t ab = __ballot(app);
    if (ab) {
        int leader = __ffsll((unsigned long long)ab) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&S.n_nxt, (uint32_t)__popcll(ab));
        base = __shfl(base, leader, 64);
        if (app) {
            uint32_t idx = base + lanes_below(ab);
            if (idx < (uint32_t)Unit2Shape<U>::FRONT) {
                S.nxt_slot[idx] = (uint16_t)h;
                S.nxt_begin[idx] = rc.begin;
                S.nxt_deg[idx] = rc.deg;
            } else {
                S.spill = 1;
            }
        }
    }
}

// expand cur entries [base, base + k) whose row begins/degrees are in cur_begin/cur_deg
template <int U>
__device__ __forceinline__ void unit2_expand(const DevGraph &g, const FRec *frec, Unit2Shared<U> &S,
                                             const uint32_t *begin, const uint32_t *deg, const uint16_t *mask,
                                             uint32_t k, uint64_t *flag_word, int shift, uint64_t &rows,
                                             uint64_t &edges) {
    uint32_t d = 0;
    if ((uint32_t)threadIdx.x < k) d = deg[threadIdx.x];
    uint32_t total = block_excl_scan2<U>(d, S);
    for (uint32_t base = 0; base < total; base += kBlock) {
        uint32_t e = base + threadIdx.x;
        bool want = e < total;
        FRec rc{0, 0, 0, 0};
        uint32_t m = 0;
        if (want) {
            uint32_t lo = 0, hi = k;  // largest j with c_pre[j] <= e
            while (hi - lo > 1) {
                uint32_t mid = (lo + hi) >> 1;
                if (S.c_pre[mid] <= e)
                    lo = mid;
                else
                    hi = mid;
            }
            rc = frec[(uint64_t)begin[lo] + (e - S.c_pre[lo])];
            m = mask[lo];
            edges++;
        }
        unit2_push<U>(g, S, want, rc, m, flag_word, shift);
    }
}

// One unit (requests [U*unit, U*unit+U)) by the whole workgroup.
template <int U>
__device__ __forceinline__ void unit2_unit(Unit2Shared<U> &S, const DevGraph &g, const FRec *frec,
                                           const uint32_t *roots, const uint32_t *targets, uint64_t n,
                                           uint64_t *allowed, uint64_t *flags, const uint64_t unit,
                                           uint32_t *spill_out, unsigned int *spill_count, unsigned long long *stats,
                                           unsigned long long *stamp) {
    const int tid = threadIdx.x;
    uint32_t n_levels = 0;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();
    const uint64_t c0 = unit * U;
    uint64_t *flag_word = &flags[c0 >> 6];
    const int shift = (int)(c0 & 63);
    const unsigned long long unit_bits = ((1ull << U) - 1) << shift;
    for (int i = tid; i < Unit2Shape<U>::H; i += kBlock) {
        S.key[i] = kEmpty;
        S.st[i] = 0;
    }
    if (tid == 0) {
        S.n_used = S.n_nxt = S.spill = S.res = S.n_hub = 0;
        S.cnt_rows = S.cnt_edges = S.cnt_rev = 0;
    }
    uint64_t rows = 0, edges = 0, rev = 0;
    if (tid < U) {  // (the same wave as tid 0: its initialization above is visible here)
        // the request, its root row (seed) and its reverse row (pull): independent loads
        uint64_t c = c0 + tid;
        uint32_t r = KETOGPU_NODE_NONE, t = KETOGPU_NODE_NONE;
        if (c < n) {
            r = roots[c];
            t = targets[c];
        }
        if (t == KETOGPU_NODE_NONE) r = KETOGPU_NODE_NONE;
        uint64_t fb = 0, fe = 0, rb = 0, re = 0;
        if (r != KETOGPU_NODE_NONE && r < kDynBase) {
            fb = g.fint_off[r];
            fe = g.fint_off[r + 1];
            rb = g.rev_off[t];
            re = g.rev_off[t + 1];
            rows += 2;
            if (g.row_amb && bit_of(g.row_amb, r))
                atomicOr((unsigned long long *)flag_word, (unsigned long long)1 << (shift + tid));
            const uint32_t hid = g.hub_mask ? g.hub_of[r] : KETOGPU_NODE_NONE;
            if (hid != KETOGPU_NODE_NONE) {  // X(r) of a hub root is its closure: nothing to expand
                fe = fb;
                uint32_t j = atomicAdd(&S.n_hub, 1u);
                if (j < (uint32_t)Unit2Shape<U>::HUBS) {
                    S.hub_id[j] = hid;
                    S.hub_slot[j] = 0xFFFF;
                    S.hub_bits[j] = (uint16_t)(1u << tid);
                } else {
                    S.spill = 1;
                }
            }
        }
        if (r != KETOGPU_NODE_NONE && r >= kDynBase) S.spill = 1;
        S.root[tid] = r;
        S.target[tid] = t;
        S.cur_begin[tid] = (uint32_t)fb;
        S.cur_deg[tid] = (uint32_t)(fe - fb);
        S.cur_mask[tid] = (uint16_t)(1u << tid);
        S.rev_b[tid] = rb;
        S.rev_n[tid] = (uint32_t)(re - rb);
    }
    __syncthreads();
    if (S.spill) {
        if (tid == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        return;
    }
    // reverse-row prefetch: issued now, stored after the seed level
    const int rj = tid / (kBlock / U), rl = tid % (kBlock / U);
    uint32_t rv = 0;
    const bool rpre = rl < kRevCache && (uint32_t)rl < S.rev_n[rj] && S.root[rj] != KETOGPU_NODE_NONE;
    if (rpre) rv = g.rev_col[S.rev_b[rj] + rl];
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();
    unit2_expand<U>(g, frec, S, S.cur_begin, S.cur_deg, S.cur_mask, U, flag_word, shift, rows, edges);
    if (rpre) S.rev_c[rj][rl] = rv;
    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();
    for (;;) {
        __syncthreads();
        uint32_t cnt = S.n_nxt;
        if (S.spill || !cnt) break;
        n_levels++;
        for (uint32_t i = tid; i < cnt; i += kBlock) {
            uint16_t s = S.nxt_slot[i];
            S.cur_slot[i] = s;
            S.cur_mask[i] = (uint16_t)(atomicAnd(&S.st[s], 0xFFFFu) >> 16);
            S.cur_begin[i] = S.nxt_begin[i];
            S.cur_deg[i] = S.nxt_deg[i];
        }
        __syncthreads();
        if (tid == 0) S.n_nxt = 0;
        for (uint32_t base = 0; base < cnt; base += kChunk) {
            uint32_t k = cnt - base < (uint32_t)kChunk ? cnt - base : (uint32_t)kChunk;
            unit2_expand<U>(g, frec, S, S.cur_begin + base, S.cur_deg + base, S.cur_mask + base, k, flag_word, shift,
                            rows, edges);
            __syncthreads();
        }
    }
    if (S.spill) {
        if (tid == 0) {
            spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
            atomicAnd((unsigned long long *)flag_word, ~unit_bits);
        }
        return;
    }
    if (stamp) stamp[3] = __builtin_amdgcn_s_memtime();
    // pull: kBlock / U lanes per request; cached reverse entries first
    {
        constexpr int L = kBlock / U;
        bool ok = false;
        uint32_t r = S.root[rj];
        if (r != KETOGPU_NODE_NONE) {
            uint32_t nrev = S.rev_n[rj];
            for (uint32_t p = rl; p < nrev && !ok; p += L) {
                uint32_t v = p < (uint32_t)kRevCache ? S.rev_c[rj][p] : g.rev_col[S.rev_b[rj] + p];
                rev++;
                if (v == r) {
                    ok = true;
                } else if (v < g.Ni) {
                    int s = key_lookup_l<Unit2Shape<U>::HLOG>(S.key, v);
                    ok = s >= 0 && ((S.st[s] >> rj) & 1u);
                    // v in the closure of a hub this request reached
                    for (uint32_t j = 0, nh = S.n_hub; j < nh && !ok; j++) {
                        const uint32_t hs = S.hub_slot[j];
                        const uint32_t bits = hs == 0xFFFFu ? S.hub_bits[j] : S.st[hs];
                        if ((bits >> rj) & 1u) {
                            const uint32_t hid = S.hub_id[j];
                            ok = (g.hub_mask[(size_t)v * g.hub_words + (hid >> 6)] >> (hid & 63)) & 1ull;
                        }
                    }
                }
            }
        }
        if (ok) atomicOr(&S.res, 1u << rj);
    }
    wave_stats_add(rows, edges, rev, &S.cnt_rows, &S.cnt_edges, &S.cnt_rev);
    __syncthreads();
    if (stamp) {
        stamp[4] = __builtin_amdgcn_s_memtime();
        stamp[5] = n_levels;
        stamp[6] = S.n_used;
        stamp[7] = 1;
    }
    if (tid == 0) {
        if (S.res) atomicOr((unsigned long long *)&allowed[c0 >> 6], (unsigned long long)S.res << shift);
        atomicAdd(&stat_slot(stats)[0], S.cnt_rows);
        atomicAdd(&stat_slot(stats)[1], S.cnt_edges);
        atomicAdd(&stat_slot(stats)[2], S.cnt_rev);
    }
}

// Pass 1 (parents == nullptr): unit b = requests [U*b, U*b+U).  Later passes split the
// spilled units of the previous pass (size U*fan) into `fan` units each.
template <int U>
__global__ __launch_bounds__(kBlock) void unit2_kernel(DevGraph g, const FRec *frec, const uint32_t *roots,
                                                       const uint32_t *targets, uint64_t n, uint64_t *allowed,
                                                       uint64_t *flags, const uint32_t *parents, uint32_t fan,
                                                       uint32_t *spill_out, unsigned int *spill_count,
                                                       unsigned long long *stats, unsigned long long *stamps) {
    __shared__ Unit2Shared<U> S;
    unsigned long long *stamp =
        (stamps && blockIdx.x < 65536 && threadIdx.x == 0) ? stamps + (size_t)blockIdx.x * 16 : nullptr;
    const uint64_t unit = parents ? (uint64_t)parents[blockIdx.x / fan] * fan + blockIdx.x % fan : blockIdx.x;
    unit2_unit<U>(S, g, frec, roots, targets, n, allowed, flags, unit, spill_out, spill_count, stats, stamp);
}

// The cascade's later stages, persistent: every unit the previous stage spilled (its count
// read on the device, so no host synchronization between stages) splits into `fan` units.
template <int U>
__global__ __launch_bounds__(kBlock) void unit2_cascade_kernel(DevGraph g, const FRec *frec, const uint32_t *roots,
                                                               const uint32_t *targets, uint64_t n, uint64_t *allowed,
                                                               uint64_t *flags, const uint32_t *parents,
                                                               const unsigned int *in_count, uint32_t fan,
                                                               uint32_t *spill_out, unsigned int *spill_count,
                                                               unsigned long long *stats) {
    __shared__ Unit2Shared<U> S;
    const uint64_t cnt = (uint64_t)*in_count * fan;
    for (uint64_t b = blockIdx.x; b < cnt; b += gridDim.x) {
        const uint64_t unit = (uint64_t)parents[b / fan] * fan + b % fan;
        unit2_unit<U>(S, g, frec, roots, targets, n, allowed, flags, unit, spill_out, spill_count, stats, nullptr);
        __syncthreads();
    }
}

// --------------------------------------------- bidirectional units (v3, default)
// Reachability is symmetric under edge reversal: with B(t) = expandable nodes that reach
// t through >= 1 edge, allowed(r, t) <=> r in B(t).  v3 grows BOTH sides of every request
// of a unit in one LDS table whose 64-bit state word per node holds, per direction d
// (0 forward, 1 backward), visited bits << 32d and pending bits << 32d + 16:
//   * forward from r over the interior subgraph (FRec records, as v2),
//   * backward from t over interior predecessors (BRec records parallel to rev_col: node
//     ids put interior nodes first and reverse rows are sorted, so a node's interior
//     predecessors are exactly the prefix of its reverse row).
// Seeds: r is forward-visited at distance 0, t backward-visited at distance 0 (unless
// t = r: a meet needs >= 1 edge).  When both seed rows are short (fint(r) and rev(t) <=
// kSeedBothMax) both are pushed at once; otherwise r and t become pending and the first
// level reads only the cheaper row, so a long rev(t) (a user with many direct grants)
// never floods the table.  A request is allowed as soon as one node carries both of its
// bits (a source entry of rev(t) can only meet r itself, so it is compared, not stored).
// Each level, every open request expands both sides while both pending degree sums are
// small, else the cheaper side (bidirectional BFS): work is bounded by the cheaper side
// and positives stop where the searches meet.  Closure: a request whose pending frontier
// is empty on one side is decided once the OTHER side's seed row has been read — every
// path r -> v1 -> ... -> v(k-1) -> t has v1 in fint(r) and v(k-1) in rev(t); if that
// seed is still pending it is expanded in lookup-only mode (checked against the closed
// side, nothing inserted).  No depth cutoff (R2).  Used when the snapshot has no
// ambiguous keys (R4 flags are raised by forward rows) and record begins fit u32;
// dynamic roots and table/list overflow spill to the next stage.
// Dead ends are looked up, not stored: a node with no interior predecessors is forward-
// visited only as r or as an entry of r's own row, and a node with no interior successors
// is backward-visited only as t or as an entry of t's own reverse row; so once the other
// side's seed row has been read (in an earlier level: its inserts are complete), a push
// of such a node only looks it up.  Leaf groups (only subject-ID members) take no slot.
// KETO_PACK=1 (default): pending-list entries pack slot, direction and degree into one
// word and the eager seed rows reuse list 1, 8,864 instead of 9,696 B of LDS per unit
// and 81 instead of 97 VGPRs: 18 instead of 16 units per CU (config #2: 0.375 vs 0.400
// ms per 10^6 requests, profiles/r02/ab_pack)
#ifndef KETO_PACK
#define KETO_PACK 1
#endif
// pending-list entries of the first-stage shape (bidi_kernel<16, 9, KETO_F1, 64, 7>)
#ifndef KETO_F1
#define KETO_F1 128
#endif
constexpr uint32_t kBothMax = 12;      // both sides expand while both pending sums are <= this
constexpr uint32_t kSeedBothMax = 32;  // seeds pushed eagerly when both seed rows are <= this

// HLOG: log2 of the LDS table slots; F: pending list capacity; BT: threads per unit
// (256 = four waves, 64 = one wave: more units per CU, barriers of one wave); LF:
// maximum table load in eighths (a unit spills beyond it)
template <int U, int HLOG, int F, int BT, int LF = 6>
struct BidiShared {
    static constexpr int H = 1 << HLOG;
    static constexpr int HMAX = H * LF / 8;
    static constexpr int EM = BT > 2 * U ? BT : 2 * U;
    alignas(16) uint32_t key[H];
    alignas(16) unsigned long long st[H];
#if KETO_PACK
    // pending lists (ping-pong): slot | dir << 15 | deg << 16 (a row of more than 65535
    // entries spills the unit), and the row's first record; the eager seed rows of the
    // first expansion use list 1 (empty until the first level appends to it)
    uint32_t p_sdd[2][F];
    uint32_t p_begin[2][F];
#else
    uint16_t p_sd[2][F];  // pending lists (ping-pong): slot | dir << 15
    uint32_t p_begin[2][F], p_deg[2][F];
    uint16_t e_sd[2 * U];  // eager seed rows: forward of r_j, backward of t_j
    uint32_t e_begin[2 * U], e_deg[2 * U];
#endif
    uint16_t e_mask[EM];   // request bits of the entries being expanded
    // block scan (BT > 64: c_pre[BT] total, wave_sum) or owner map (one wave: c_pre[64])
    uint32_t c_pre[BT > 64 ? BT + 1 : BT];
    uint32_t wave_sum[BT > 64 ? BT / 64 : 1];
    uint32_t cost[2][U];          // pending degree sums per direction and request
    uint32_t root[U];
    uint32_t sel[2], lookup[2];   // per direction: bits expanded this level / lookup-only bits
    uint32_t sread[2];            // per direction: bits for which a push of a dead-end node is lookup-only
    uint32_t n_used, n_p[2], spill, found, active;
    // unit statistics (workgroups of several waves; one wave adds its own to the global slots)
    unsigned long long cnt[BT > 64 ? 3 : 1];
};

// per-level selection, wave-uniform: open requests, bits expanded per direction, lookup-only
// bits, and bits for which a dead-end push is lookup-only (one-wave units keep it in SGPRs)
struct BidiLevel {
    uint32_t active;
    uint32_t sel[2], lookup[2], sread[2];
};

// exclusive block scan of one u32 per thread (BT threads) into S.c_pre; returns the total
template <int BT, class SH>
__device__ __forceinline__ uint32_t block_scan_sh(uint32_t v, SH &S) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
    }
    if (lane == 63) S.wave_sum[wv] = x;
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int i = 0; i < BT / 64; i++) {
        uint32_t s = S.wave_sum[i];
        base += i < wv ? s : 0;
        total += s;
    }
    S.c_pre[tid] = base + x - v;
    if (tid == 0) S.c_pre[BT] = total;
    __syncthreads();
    return total;
}

// one wave's LDS writes visible to its own later reads (a workgroup of several waves whose
// waves work on their own data)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wave-aggregated append to an LDS list: index of this lane's entry (all lanes call)
__device__ __forceinline__ uint32_t lds_append(bool want, uint32_t *counter) {
    uint64_t bal = __ballot(want);
    uint32_t base = 0;
    if (bal) {
        int leader = __ffsll((unsigned long long)bal) - 1;  // wave-uniform
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, (uint32_t)__popcll(bal));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);  // v_readlane, not an LDS permute
    }
    return base + lanes_below(bal);
}

// find (insert == false) or find-or-insert u; -1 when absent (or the table is full)
template <int HLOG>
__device__ __forceinline__ int bidi_slot(uint32_t *key, uint32_t u, bool insert, bool &inserted) {
    constexpr int H = 1 << HLOG;
    uint32_t hh = (u * 2654435761u) >> (32 - HLOG);
#if KETO_PROBE_ROLLED
#pragma unroll 1
#endif
    for (int p = 0; p < H; p++, hh = (hh + 1) & (H - 1)) {
        // insert: compare-and-swap first (one LDS round trip per probe, whether the slot
        // is empty, holds u or holds another key)
        const uint32_t kv = insert ? atomicCAS(&key[hh], kEmpty, u) : key[hh];
        if (kv == kEmpty) {
            if (!insert) return -1;
            inserted = true;
            return (int)hh;
        }
        if (kv == u) return (int)hh;
    }
    return -1;
}

// Pending degree sums: cost[d][j] += (sub ? -1 : 1) * sum over the wave's lanes whose
// `bits` hold request j, in direction d, of `val`.  Called by every lane of the wave.
// KETO_COST_ATOMIC=1 (default): one LDS atomic per lane and bit.  KETO_COST_ATOMIC=0: the
// wave reduces each (direction, request) sum with DPP and one lane updates it — fewer LDS
// bank conflicts, but measured 1.5x slower on config #2 (0.618 vs 0.405 ms per 1M
// requests): the reductions cost more VALU/SALU issue than the conflicts they remove.
#ifndef KETO_COST_ATOMIC
#define KETO_COST_ATOMIC 1  // measured: per-lane atomics 0.405 ms, the wave reductions 0.618 ms per 1M requests
#endif
#if !KETO_COST_ATOMIC
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 15) | __builtin_amdgcn_readlane((int)x, 31) |
                      __builtin_amdgcn_readlane((int)x, 47) | __builtin_amdgcn_readlane((int)x, 63));
}
#endif

template <int BT, class SH>
__device__ __forceinline__ void cost_update(SH &S, uint32_t bits, int d, uint32_t val, bool sub) {
#if KETO_COST_ATOMIC
    for (uint32_t b = bits; b; b &= b - 1) {
        if (sub)
            atomicSub(&S.cost[d][__ffs(b) - 1], val);
        else
            atomicAdd(&S.cost[d][__ffs(b) - 1], val);
    }
#else
    const int lane = threadIdx.x & 63;
    for (int dd = 0; dd < 2; dd++) {
        const uint32_t mine = d == dd ? bits : 0u;
        uint32_t any = wave_or_u32(mine);  // wave-uniform
        while (any) {
            const int j = __ffs(any) - 1;
            any &= any - 1;
            const uint32_t v = (mine >> j) & 1u ? val : 0u;
            const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_u32(v), 63);
            if (lane == 0) {
                if constexpr (BT == 64) {
                    S.cost[dd][j] = sub ? S.cost[dd][j] - sum : S.cost[dd][j] + sum;
                } else if (sub) {
                    atomicSub(&S.cost[dd][j], sum);
                } else {
                    atomicAdd(&S.cost[dd][j], sum);
                }
            }
        }
    }
#endif
}

// Push mask m into node u in direction d.  Bits in L.lookup[d] belong to requests whose
// other side is closed: for them u is only looked up (a meet or nothing), never inserted
// nor made pending.  New pending bits add deg to their requests' pending sums.
template <int U, int HLOG, int F, int BT, int LF>
__device__ __forceinline__ void bidi_push(BidiShared<U, HLOG, F, BT, LF> &S, const BidiLevel &L, bool want, uint32_t u,
                                          uint32_t deg, uint32_t begin, uint32_t m, int d, int nxt) {
    const uint32_t lk = m & ((d ? L.lookup[1] : L.lookup[0]) | (deg ? 0u : (d ? L.sread[1] : L.sread[0])));
    int h = -1;
    bool inserted = false;
    if (want) {
        const bool ins = (m & ~lk) != 0;
        h = bidi_slot<HLOG>(S.key, u, ins, inserted);
        if (h < 0 && ins) S.spill = 1;
    }
    const int lane = threadIdx.x & 63;
    uint64_t bal = __ballot(inserted);
    // table load: counted without a return value, compared with HMAX after the next barrier
    if (bal && lane == __ffsll((unsigned long long)bal) - 1) atomicAdd(&S.n_used, (uint32_t)__popcll(bal));
    bool app = false;
    uint32_t pend = 0;  // requests for which u becomes pending
    if (h >= 0) {
        const int vs = 32 * d;
        // one 64-bit atomic per push: the old word also carries the other direction's
        // visited bits, so of two pushes that complete a meet the later one sees it
        unsigned long long old = atomicOr(&S.st[h], (unsigned long long)m << vs);
        uint32_t newly = m & ~(uint32_t)(old >> vs) & 0xFFFFu;
        uint32_t meet = newly & (uint32_t)(old >> (32 - vs)) & 0xFFFFu;
        if (meet) atomicOr(&S.found, meet);
        newly &= ~(meet | lk);
        if (newly && deg) {
            unsigned long long o2 = atomicOr(&S.st[h], (unsigned long long)newly << (vs + 16));
            app = !((uint32_t)(o2 >> (vs + 16)) & 0xFFFFu);
            pend = newly;
        }
    }
    cost_update<BT>(S, pend, d, deg, false);
    uint32_t idx = lds_append(app, &S.n_p[nxt]);
    if (app) {
#if KETO_PACK
        if (idx < (uint32_t)F && deg <= 0xFFFFu) {
            S.p_sdd[nxt][idx] = (uint32_t)h | ((uint32_t)d << 15) | (deg << 16);
            S.p_begin[nxt][idx] = begin;
        } else {
            S.spill = 1;
        }
#else
        if (idx < (uint32_t)F) {
            S.p_sd[nxt][idx] = (uint16_t)(h | (d << 15));
            S.p_begin[nxt][idx] = begin;
            S.p_deg[nxt][idx] = deg;
        } else {
            S.spill = 1;
        }
#endif
    }
}

// one source predecessor u of t (u >= Ni): it meets only r itself, so it is compared with
// the requests' roots instead of being stored
template <int U, int HLOG, int F, int BT, int LF>
__device__ __forceinline__ void bidi_source_meet(BidiShared<U, HLOG, F, BT, LF> &S, uint32_t u, uint32_t m) {
    uint32_t hit = 0;
    for (uint32_t b = m; b; b &= b - 1)
        if (S.root[__ffs(b) - 1] == u) hit |= b & (~b + 1);
    if (hit) atomicOr(&S.found, hit);
}

// One-wave units (BT == 64): entry j on lane j (k <= 64).  Register scan of the degrees, an
// owner map per 64-edge chunk (each entry that overlaps the chunk writes its index at its
// first position in it — positions are distinct — and a prefix maximum fills the gaps;
// positions a chunk does not write hold owners of earlier edges, never larger), and the
// record loads software-pipelined one chunk ahead of the pushes.
template <int U, int HLOG, int F, int BT, int LF, class SDT>
__device__ __forceinline__ void bidi_expand64(const DevGraph &g, const FRec *frec, const FRec *brec,
                                              BidiShared<U, HLOG, F, BT, LF> &S, const BidiLevel &L, uint32_t my_deg,
                                              const SDT *sd, const uint32_t *begin, int nxt, uint64_t &edges) {
    const uint32_t lane = threadIdx.x;
    const uint32_t incl = wave_incl_sum_u32(my_deg);
    const uint32_t start = incl - my_deg;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (!total) return;
    S.c_pre[lane] = 0xFFFFFFFFu;
    struct Edge {
        uint32_t lo;  // owning entry
        uint32_t ls;  // its first edge
        int d;        // its direction
        FRec rc;      // the record of edge eb + lane
    };
    // Owner of edge eb + lane, then its record.  `more` false: no chunk at eb — the load is
    // still issued (the previous chunk's edge again, an L2 hit), because a load under a
    // branch is merged by a register copy that waits for it right away.
    auto fetch = [&](uint32_t eb, Edge &x, bool more, const Edge &prev) {
        uint32_t e;
        if (more) {
            if (my_deg && start < eb + 64 && start + my_deg > eb) S.c_pre[(start > eb ? start : eb) - eb] = lane;
            __syncthreads();
            const int o = wave_incl_max_i32((int)S.c_pre[lane]);
            x.lo = (uint32_t)(o < 0 ? 0 : o);
            x.ls = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x.lo << 2), (int)start);
            x.d = (int)((uint32_t)(sd[x.lo] >> 15) & 1u);
            e = min(eb + lane, total - 1);  // lanes past the end re-read the last edge
        } else {
            x.lo = prev.lo;
            x.ls = prev.ls;
            x.d = prev.d;
            e = min(eb - 64 + lane, total - 1);
        }
        x.rc = (x.d ? brec : frec)[(uint64_t)begin[x.lo] + (e - x.ls)];
    };
    auto push = [&](uint32_t eb, const Edge &x) {
        uint32_t m = 0;
        if (eb + lane < total) {
            m = S.e_mask[x.lo] & L.active & ~S.found;
            edges++;
            if (x.d && x.rc.node >= g.Ni) {
                bidi_source_meet<U, HLOG, F, BT, LF>(S, x.rc.node, m);
                m = 0;
            }
        }
        bidi_push<U, HLOG, F, BT, LF>(S, L, m != 0, x.rc.node, x.rc.deg, x.rc.begin, m, x.d, nxt);
    };
    // two register sets in turn, so the next chunk's loads fly during this chunk's pushes
    // without a loop-carried copy
    Edge a{}, b{};
    fetch(0, a, true, b);
    for (uint32_t eb = 0;;) {
        const bool more = eb + 64 < total;  // wave-uniform
        fetch(eb + 64, b, more, a);
        push(eb, a);
        if (!more) break;
        eb += 64;
        const bool more2 = eb + 64 < total;
        fetch(eb + 64, a, more2, b);
        push(eb, b);
        if (!more2) break;
        eb += 64;
    }
}

// Expand k entries (entry j: sd[j], begin[j], S.e_mask[j]); `my_deg` is the degree this
// thread contributes for entry threadIdx.x (0 when it has none).  Block-uniform loop.
template <int U, int HLOG, int F, int BT, int LF, class SDT>
__device__ __forceinline__ void bidi_expand(const DevGraph &g, const FRec *frec, const FRec *brec,
                                            BidiShared<U, HLOG, F, BT, LF> &S, const BidiLevel &L, uint32_t my_deg,
                                            uint32_t k, const SDT *sd, const uint32_t *begin, int nxt,
                                            uint64_t &edges) {
    if constexpr (BT == 64) {
        bidi_expand64<U, HLOG, F, BT, LF, SDT>(g, frec, brec, S, L, my_deg, sd, begin, nxt, edges);
    } else {  // several waves: block scan + binary search for each edge's entry
        const uint32_t total = block_scan_sh<BT>(my_deg, S);
        for (uint32_t eb = 0; eb < total; eb += BT) {
            uint32_t e = eb + threadIdx.x;
            bool want = e < total;
            uint32_t u = 0, deg = 0, bg = 0, m = 0;
            int d = 0;
            if (want) {
                uint32_t lo = 0, hi = k;  // largest j with c_pre[j] <= e
                while (hi - lo > 1) {
                    uint32_t mid = (lo + hi) >> 1;
                    if (S.c_pre[mid] <= e)
                        lo = mid;
                    else
                        hi = mid;
                }
                d = (int)((uint32_t)(sd[lo] >> 15) & 1u);
                m = S.e_mask[lo] & L.active & ~S.found;
                FRec rc = (d ? brec : frec)[(uint64_t)begin[lo] + (e - S.c_pre[lo])];
                u = rc.node;
                deg = rc.deg;
                bg = rc.begin;
                edges++;
                if (d && u >= g.Ni) {
                    bidi_source_meet<U, HLOG, F, BT, LF>(S, u, m);
                    m = 0;
                }
                want = m != 0;
            }
            bidi_push<U, HLOG, F, BT, LF>(S, L, want, u, deg, bg, m, d, nxt);
        }
    }
}

// The seeds of request `threadIdx.x` of a unit (lanes < U): its root and target, then the
// offsets of both seed rows (two dependent loads).  A persistent first stage that loaded
// them one unit ahead measured slower than one workgroup per unit (static striding 0.475
// vs 0.435 ms per 1M requests: tail imbalance and 107 VGPRs; a device-scope work counter
// 0.89 ms: every record-load wait also waited for the counter's atomic).
struct BidiSeed {
    uint32_t r, t;
    uint64_t fb, fe, rb, re;
};

template <int U>
__device__ __forceinline__ void bidi_load_rt(uint64_t unit, uint64_t units, const uint32_t *roots,
                                             const uint32_t *targets, uint64_t n, uint32_t &r, uint32_t &t) {
    r = t = KETOGPU_NODE_NONE;
    const uint64_t c = unit * U + threadIdx.x;
    if (threadIdx.x < U && unit < units && c < n) {
        r = roots[c];
        t = targets[c];
    }
}

__device__ __forceinline__ BidiSeed bidi_load_rows(const DevGraph &g, uint32_t r, uint32_t t) {
    BidiSeed s{t == KETOGPU_NODE_NONE ? KETOGPU_NODE_NONE : r, t, 0, 0, 0, 0};
    if (s.r != KETOGPU_NODE_NONE && s.r < kDynBase) {
        s.fb = g.fint_off[s.r];
        s.fe = g.fint_off[s.r + 1];
        s.rb = g.rev_off[t];
        s.re = g.rev_off[t + 1];
    }
    return s;
}

// plan core: the seed rows from the node blocks (core_index.hpp) — one 16-byte header per
// row {count, first record (64 bits)} at the head of the node's block, a short row on the
// header's own cache line(s) right behind it: one dependent HBM read instead of the offset
// pair and then the records
__device__ __forceinline__ BidiSeed core_load_rows(const DevGraph &g, const FRec *frec, const FRec *brec, uint32_t r,
                                                   uint32_t t) {
    BidiSeed s{t == KETOGPU_NODE_NONE ? KETOGPU_NODE_NONE : r, t, 0, 0, 0, 0};
    if (s.r != KETOGPU_NODE_NONE && s.r < kDynBase) {
        const FRec hf = frec[g.blk[0] + ((uint64_t)s.r << g.blk_log[0])];
        const FRec hb = brec[g.blk[1] + ((uint64_t)t << g.blk_log[1])];
        s.fb = (uint64_t)hf.deg | (uint64_t)hf.begin << 32;
        s.fe = s.fb + hf.node;
        s.rb = (uint64_t)hb.deg | (uint64_t)hb.begin << 32;
        s.re = s.rb + hb.node;
    }
    return s;
}

// one unit (requests [U*unit, U*unit + U)) by the whole workgroup; `seed` as loaded by
// bidi_load_rt + bidi_load_rows on lanes < U
template <int U, int HLOG, int F, int BT, int LF>
__device__ __forceinline__ void bidi_unit(BidiShared<U, HLOG, F, BT, LF> &S, const DevGraph &g, const FRec *frec,
                                          const FRec *brec, const BidiSeed &seed, uint64_t *allowed,
                                          const uint64_t unit, uint32_t *spill_out, unsigned int *spill_count,
                                          unsigned long long *stats, unsigned long long *stamp) {
    static_assert(U <= 16, "16 request bits per direction");
    using SH = BidiShared<U, HLOG, F, BT, LF>;
    const int tid = threadIdx.x;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();
    const uint64_t c0 = unit * U;
    const int shift = (int)(c0 & 63);
    // clear the table with 16-byte stores (4 keys or 2 state words per store)
    for (int i = tid; i < SH::H / 4; i += BT) reinterpret_cast<uint4 *>(S.key)[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    for (int i = tid; i < SH::H / 2; i += BT) reinterpret_cast<uint4 *>(S.st)[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) {
        S.n_used = S.n_p[0] = S.n_p[1] = S.spill = S.found = S.active = 0;
        if constexpr (BT > 64) S.cnt[0] = S.cnt[1] = S.cnt[2] = 0;
    }
    if (tid < 2 * U) S.cost[tid / U][tid % U] = 0;
    if (tid < 2) {
        S.lookup[tid] = 0;
        S.sread[tid] = 0;
    }
    __syncthreads();
    uint64_t rows = 0, edges = 0;
    uint32_t n_levels = 0;
    int rslot = 0, tslot = 0;  // table slots of this lane's request's seeds (wave 0, lane j = request j)
    const uint32_t r = seed.r, t = seed.t;
    const uint64_t fb = seed.fb, fe = seed.fe, rb = seed.rb, re = seed.re;
    if (tid < U) {
        if (r != KETOGPU_NODE_NONE && r < kDynBase) {
            rows += 2;
            if (re > rb) atomicOr(&S.active, 1u << tid);  // nothing reaches a t without predecessors
        }
        if (r != KETOGPU_NODE_NONE && r >= kDynBase) S.spill = 1;
        S.root[tid] = r;
    }
    __syncthreads();
    if (S.spill) {
        if (tid == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        return;
    }
    if (tid < 64) {  // wave 0: lane j < U seeds request j
        const bool v = tid < U && ((S.active >> tid) & 1u);
        const uint32_t bit = 1u << (tid & 15);
        const uint32_t rdeg = (uint32_t)(fe - fb), tdeg = (uint32_t)(re - rb);
        const bool eager = rdeg <= g.seed_max && tdeg <= g.seed_max;
        for (int side = 0; side < 2; side++) {
            const uint32_t u = side ? t : r, deg = side ? tdeg : rdeg;
            bool inserted = false;
            const int h = v ? bidi_slot<HLOG>(S.key, u, true, inserted) : -1;
            uint64_t bal = __ballot(inserted);
            if (tid == 0) S.n_used += (uint32_t)__popcll(bal);  // <= 2U slots, far below HMAX
            bool app = false;
            if (h >= 0) {
                if (side == 0)
                    rslot = h;
                else
                    tslot = h;
                const bool pend = !eager && deg;
                unsigned long long bits = (side == 0 || t != r) ? (unsigned long long)bit << (32 * side) : 0ull;
                if (pend) bits |= (unsigned long long)bit << (32 * side + 16);
                unsigned long long old = atomicOr(&S.st[h], bits);
                app = pend && !((uint32_t)(old >> (32 * side + 16)) & 0xFFFFu);
                if (pend) atomicAdd(&S.cost[side][tid], deg);
            }
            uint32_t idx = lds_append(app, &S.n_p[0]);
            if (app) {  // idx < 2U <= F
#if KETO_PACK
                if (deg > 0xFFFFu) S.spill = 1;  // a seed row longer than the packed degree
                S.p_sdd[0][idx] = (uint32_t)h | ((uint32_t)side << 15) | (deg << 16);
                S.p_begin[0][idx] = (uint32_t)(side ? rb : fb);
#else
                S.p_sd[0][idx] = (uint16_t)(h | (side << 15));
                S.p_begin[0][idx] = (uint32_t)(side ? rb : fb);
                S.p_deg[0][idx] = deg;
#endif
            }
        }
        if (tid < U) {  // eager rows (zero degree when not eager or not active)
            const bool e = v && eager;
#if KETO_PACK
            S.p_sdd[1][tid] = (e ? rdeg : 0u) << 16;  // eager degrees <= seed_max (< 65536)
            S.p_begin[1][tid] = (uint32_t)fb;
            S.p_sdd[1][U + tid] = (1u << 15) | ((e ? tdeg : 0u) << 16);
            S.p_begin[1][U + tid] = (uint32_t)rb;
#else
            S.e_sd[tid] = 0;
            S.e_begin[tid] = (uint32_t)fb;
            S.e_deg[tid] = e ? rdeg : 0;
            S.e_sd[U + tid] = (uint16_t)(1u << 15);
            S.e_begin[U + tid] = (uint32_t)rb;
            S.e_deg[U + tid] = e ? tdeg : 0;
#endif
        }
        if (tid < 2 * U) S.e_mask[tid] = (uint16_t)(1u << (tid % U));
    }
    __syncthreads();
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();
    BidiLevel L{S.active, {0, 0}, {0, 0}, {0, 0}};  // the seed rows: every push inserts
#if KETO_PACK
    bidi_expand<U, HLOG, F, BT, LF>(g, frec, brec, S, L, (uint32_t)tid < 2 * U ? S.p_sdd[1][tid] >> 16 : 0, 2 * U,
                                    S.p_sdd[1], S.p_begin[1], 0, edges);
#else
    bidi_expand<U, HLOG, F, BT, LF>(g, frec, brec, S, L, (uint32_t)tid < 2 * U ? S.e_deg[tid] : 0, 2 * U, S.e_sd,
                                    S.e_begin, 0, edges);
#endif
    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();
    int cur = 0;
    bool spilled = false;
    for (;;) {
        __syncthreads();
        const uint32_t cnt = S.n_p[cur];
        const uint32_t act = L.active & ~S.found;
        if (S.spill || (S.n_used > (uint32_t)SH::HMAX && act)) {  // undecided requests, table over its load
            spilled = true;
            break;
        }
        if (!cnt || !act) break;
        n_levels++;
        unsigned long long tp0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
        const int nxt = cur ^ 1;
        if (tid < 64) {
            // per request: expand both sides while both are cheap, else the cheaper one;
            // a closed side decides the request once the other seed row has been read,
            // else that seed is read in lookup-only mode
            const bool a = tid < U && ((act >> tid) & 1u);
            const uint32_t cf = a ? S.cost[0][tid] : 0, cb = a ? S.cost[1][tid] : 0;
            const int j = tid & 15;
            const bool fc = a && !cf, bc = a && !cb;
            // seed rows still unread (only needed when a side is closed)
            const bool rpend = a && ((S.st[rslot] >> (16 + j)) & 1ull);
            const bool rp = bc && rpend;
            const bool tpend = a && ((S.st[tslot] >> (48 + j)) & 1ull);
            const bool tp = fc && tpend;
            const bool closed = (fc && !tp) || (bc && !rp) || (fc && bc);
            const bool open = a && !closed;
            const bool lkb = open && fc, lkf = open && bc;
            const bool both = open && !fc && !bc && cf <= g.both_max && cb <= g.both_max;
            const bool fwd = lkf || both || (open && !fc && !bc && cf <= cb);
            const bool bwd = lkb || both || (open && !fc && !bc && cf > cb);
            const uint64_t bcl = __ballot(closed), bf = __ballot(fwd), bb = __ballot(bwd);
            const uint64_t lf = __ballot(lkf), lb = __ballot(lkb), tr = __ballot(a && !tpend);
            const uint64_t rr = __ballot(a && !rpend);
            L = BidiLevel{act & ~(uint32_t)bcl, {(uint32_t)bf, (uint32_t)bb}, {(uint32_t)lf, (uint32_t)lb},
                          {(uint32_t)tr, (uint32_t)rr}};
            if (tid == 0) {
                if constexpr (BT > 64) {  // other waves read the selection from LDS
                    S.active = L.active;
                    S.sel[0] = L.sel[0];
                    S.sel[1] = L.sel[1];
                    S.lookup[0] = L.lookup[0];
                    S.lookup[1] = L.lookup[1];
                    S.sread[0] = L.sread[0];
                    S.sread[1] = L.sread[1];
                }
                S.n_p[nxt] = 0;
            }
        }
        __syncthreads();
        if constexpr (BT > 64)
            L = BidiLevel{S.active, {S.sel[0], S.sel[1]}, {S.lookup[0], S.lookup[1]}, {S.sread[0], S.sread[1]}};
        unsigned long long tp1 = stamp ? __builtin_amdgcn_s_memtime() : 0;
        // chunks of BT pending entries: the chosen direction's bits are taken (their
        // pending sums drop) and expanded right away, open requests' other bits stay
        // pending (the entry is carried to the next list)
        const uint32_t act2 = L.active;
        for (uint32_t base = 0; base < cnt && !S.spill && S.n_used <= (uint32_t)SH::HMAX; base += BT) {  // read after a barrier
            const uint32_t k = cnt - base < (uint32_t)BT ? cnt - base : (uint32_t)BT;
            const uint32_t i = base + tid;
            uint32_t take = 0, rest = 0, sd = 0, dg = 0, bg = 0, clr = 0;
            if ((uint32_t)tid < k) {
#if KETO_PACK
                const uint32_t w = S.p_sdd[cur][i];
                sd = w & 0xFFFFu;
                dg = w >> 16;
#else
                sd = S.p_sd[cur][i];
                dg = S.p_deg[cur][i];
#endif
                bg = S.p_begin[cur][i];
                const uint32_t d = sd >> 15, s = sd & 0x7FFFu;
                const uint32_t pb = (uint32_t)(S.st[s] >> (32 * d + 16)) & 0xFFFFu;
                take = pb & (d ? L.sel[1] : L.sel[0]);
                rest = pb & act2 & ~take;
                clr = pb & ~rest;
                if (clr) atomicAnd(&S.st[s], ~((unsigned long long)clr << (32 * d + 16)));
                S.e_mask[tid] = (uint16_t)take;
            }
            cost_update<BT>(S, clr, (int)(sd >> 15), dg, true);
            const uint32_t pi = lds_append(rest != 0, &S.n_p[nxt]);
            if (rest) {
                if (pi < (uint32_t)F) {
#if KETO_PACK
                    S.p_sdd[nxt][pi] = sd | (dg << 16);
#else
                    S.p_sd[nxt][pi] = (uint16_t)sd;
                    S.p_deg[nxt][pi] = dg;
#endif
                    S.p_begin[nxt][pi] = bg;
                } else {
                    S.spill = 1;
                }
            }
#if KETO_PACK
            bidi_expand<U, HLOG, F, BT, LF>(g, frec, brec, S, L, take ? dg : 0, k, S.p_sdd[cur] + base,
                                            S.p_begin[cur] + base, nxt, edges);
#else
            bidi_expand<U, HLOG, F, BT, LF>(g, frec, brec, S, L, take ? dg : 0, k, S.p_sd[cur] + base,
                                            S.p_begin[cur] + base, nxt, edges);
#endif
            __syncthreads();
        }
        if (stamp) {
            unsigned long long tp2 = __builtin_amdgcn_s_memtime();
            stamp[8] += tp1 - tp0;
            stamp[11] += tp2 - tp1;
        }
        cur = nxt;
    }
    __syncthreads();
    if (spilled || S.spill) {
        if (tid == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        return;
    }
    if (stamp) stamp[3] = __builtin_amdgcn_s_memtime();
    if constexpr (BT > 64) {
        wave_stats_add(rows, edges, 0, &S.cnt[0], &S.cnt[1], &S.cnt[2]);
        __syncthreads();
    } else {  // one wave: its sums go straight to the global slots
#pragma unroll
        for (int s = 32; s; s >>= 1) {
            rows += __shfl_down(rows, s, 64);
            edges += __shfl_down(edges, s, 64);
        }
    }
    if (stamp) {
        stamp[4] = stamp[3];
        stamp[5] = n_levels;
        stamp[6] = S.n_used;
        stamp[7] = 1;
    }
    if (tid == 0) {
        uint32_t res = S.found & ((1u << U) - 1);
        if (res) atomicOr((unsigned long long *)&allowed[c0 >> 6], (unsigned long long)res << shift);
        atomicAdd(&stat_slot(stats)[0], BT > 64 ? S.cnt[0] : (unsigned long long)rows);
        atomicAdd(&stat_slot(stats)[1], BT > 64 ? S.cnt[1] : (unsigned long long)edges);
    }
}

// Stage kernel.  in_count == nullptr: workgroup b runs unit parents ? parents[b] : unit0 + b.
// Otherwise persistent: the workgroups stride over the *in_count units listed in
// parents (the previous stage's spills), so the stage is launched without the host
// reading that count first.
// WPE > 1 asks the compiler for at least WPE waves per SIMD (VGPR budget 512 / WPE): with
// 5 KB of LDS, 8-request units could run 32 per CU at WPE 8
// CHUNKED = 1: the same kernel for the pipelined host-to-host first stage (check_host),
// one launch per chunk; a separate symbol keeps its launches apart in kernel traces.
template <int U, int HLOG, int F, int BT, int LF, int WPE = 1, int CHUNKED = 0>
__global__ __launch_bounds__(BT) __attribute__((amdgpu_waves_per_eu(WPE)))
void bidi_kernel(DevGraph g, const FRec *frec, const FRec *brec,
                                                  const uint32_t *roots, const uint32_t *targets, uint64_t n,
                                                  uint64_t *allowed, const uint32_t *parents,
                                                  const unsigned int *in_count, uint32_t fan, uint32_t *spill_out,
                                                  unsigned int *spill_count, unsigned long long *stats,
                                                  unsigned long long *stamps, uint64_t unit0) {
    __shared__ BidiShared<U, HLOG, F, BT, LF> S;
    const uint64_t units = (n + U - 1) / U;
    if (!in_count) {
        unsigned long long *stamp =
            (stamps && blockIdx.x < 65536 && threadIdx.x == 0) ? stamps + (size_t)blockIdx.x * 16 : nullptr;
        // unit0: a pipelined batch launches its units chunk by chunk, as each chunk of
        // requests arrives in HBM (ketogpu_engine::check_host)
        const uint64_t unit = parents ? parents[blockIdx.x] : unit0 + blockIdx.x;
        uint32_t r, t;
        bidi_load_rt<U>(unit, units, roots, targets, n, r, t);
        bidi_unit<U, HLOG, F, BT, LF>(S, g, frec, brec, bidi_load_rows(g, r, t), allowed, unit, spill_out,
                                      spill_count, stats, stamp);
        return;
    }
    // persistent: every listed unit of the previous stage splits into `fan` units of U
    const uint64_t cnt = (uint64_t)*in_count * fan;
    for (uint64_t b = blockIdx.x; b < cnt; b += gridDim.x) {
        const uint64_t unit = (uint64_t)parents[b / fan] * fan + b % fan;
        uint32_t r, t;
        bidi_load_rt<U>(unit, units, roots, targets, n, r, t);
        bidi_unit<U, HLOG, F, BT, LF>(S, g, frec, brec, bidi_load_rows(g, r, t), allowed, unit, spill_out,
                                      spill_count, stats, nullptr);
        __syncthreads();
    }
}

// Host-to-host first stage in ONE launch (ketogpu_engine::check_host, pinned requests):
// each unit reads its 16 roots and targets straight from pinned host memory over PCIe
// (128 B per unit, ~8 MB per 10^6 requests spread over the whole traversal), validates
// them as validate_kernel does and stores them in HBM for the spill stages.  Replaces
// the chunk pipeline (load_kernel per chunk + one first-stage launch per chunk on two
// streams): no exposed first-chunk upload, one launch tail instead of one per chunk.
// K units per workgroup, run one after the other: the requests of all K are read at the
// start, so only the first unit waits for PCIe (a read from host memory takes several
// times an HBM miss and every unit would wait for one).
// The requests of a host-batch workgroup's K 16-request units, read in place from pinned
// host memory over PCIe, returned on lanes < 16 (unit k: r[k], t[k]); ids outside the
// snapshot are reported (first_bad) and become NONE; the validated ids go to HBM (dr, dt)
// for the spill stages.  Every lane reads: a workgroup's 16K roots and 16K targets are two
// contiguous runs of 64K bytes, so K = 1 / 2 take ONE wave instruction (roots on lanes
// 0-31, targets on lanes 32-63) and K = 4 two of 256 contiguous bytes each — instead of
// 2K instructions of 64 bytes (the in-kernel PCIe reads then ran at ~36 GB/s).
template <int K>
__device__ __forceinline__ void host_unit_requests(const DevGraph &g, const uint32_t *hr, const uint32_t *ht,
                                                   uint32_t *dr, uint32_t *dt, uint64_t n,
                                                   unsigned long long *first_bad, uint32_t (&r)[K], uint32_t (&t)[K]) {
    static_assert(K == 1 || K == 2 || K == 4, "1, 2 or 4 units per workgroup");
    const uint32_t lane = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * K * 16;
    uint32_t vr = KETOGPU_NODE_NONE, vt = KETOGPU_NODE_NONE;
    if constexpr (K == 4) {
        if (base + lane < n) {
            vr = hr[base + lane];
            vt = ht[base + lane];
        }
    } else {
        const uint32_t j = lane & 31;
        if (j < 16 * K && base + j < n) vr = (lane < 32 ? hr : ht)[base + j];
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int src = 16 * k + (int)(lane & 15);
        r[k] = (uint32_t)__shfl((int)vr, src, 64);
        t[k] = (uint32_t)__shfl((int)(K == 4 ? vt : vr), K == 4 ? src : 32 + src, 64);
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t c = base + 16 * k + lane;
        if (lane < 16 && c < n) {
            if ((r[k] != KETOGPU_NODE_NONE && r[k] >= g.Nx) || (t[k] != KETOGPU_NODE_NONE && t[k] >= g.N)) {
                atomicMin(first_bad, (unsigned long long)c);
                r[k] = t[k] = KETOGPU_NODE_NONE;
            }
            dr[c] = r[k];
            dt[c] = t[k];
        }
    }
}

template <int K>
__global__ __launch_bounds__(64) void bidi_host_kernel(DevGraph g, const FRec *frec, const FRec *brec,
                                                       const uint32_t *hr, const uint32_t *ht, uint32_t *dr,
                                                       uint32_t *dt, uint64_t n, uint64_t *allowed, uint32_t *spill_out,
                                                       unsigned int *spill_count, unsigned long long *stats,
                                                       unsigned long long *first_bad) {
    __shared__ BidiShared<16, 9, KETO_F1, 64, 7> S;
    uint32_t r[K], t[K];
    host_unit_requests<K>(g, hr, ht, dr, dt, n, first_bad, r, t);
    const uint64_t units = (n + 15) / 16;
#pragma unroll 1
    for (int k = 0; k < K; k++) {
        const uint64_t unit = (uint64_t)blockIdx.x * K + k;
        if (unit >= units) break;
        uint32_t rk = r[0], tk = t[0];
#pragma unroll
        for (int j = 1; j < K; j++)
            if (j == k) rk = r[j], tk = t[j];
        // (loading every unit's seed-row offsets up front as well measured slower: 1.99
        // vs 2.10 x 10^9 checks/s, profiles/r02/ab_prerows)
        const BidiSeed sk = bidi_load_rows(g, rk, tk);
        bidi_unit<16, 9, KETO_F1, 64, 7>(S, g, frec, brec, sk, allowed, unit, spill_out, spill_count, stats, nullptr);
        __syncthreads();
    }
}

// ----------------------------------------------------------------------- bidi-lite
// The first stage of plan "lite" (round 3): the bidirectional meet of bidi_kernel with the
// per-request bookkeeping taken out of the hot loop.  Counters of the round-2 kernel put
// its instruction issue, not HBM, at the limit (VALU issue 63%, 2,261 VALU + 1,617 SALU
// per 16-request unit for ~305 edges), and most of those instructions were
// per-level overhead: per-request pending-degree sums kept with one LDS atomic per lane
// and request bit on every push and every take (39% of LDS cycles in bank conflicts on
// the 32-word cost array), per-request direction choice that split every pending entry
// into taken and carried parts, and a per-level selection over LDS state.  Here:
//   * the DIRECTION is chosen per unit and level: both sides while both pending degree
//     totals are small, else the side with the smaller total (sums accumulated in lane
//     registers during the pushes, one wave reduction per level);
//   * every direction has its own ring of pending rows, consumed whole when that
//     direction is expanded (one LDS atomic reads and clears an entry's pending bits);
//   * per-request closure is pure SGPR bit logic on 16-bit masks: pf / pb = requests with
//     a pending row in the forward / backward ring (OR of the pushes' new pending bits,
//     one reduction per level), rpend / tpend = requests whose own seed row is still
//     unread.  A request is decided false when one side has nothing pending and the other
//     side's seed row has been read (every path r -> v1 -> ... -> t has v1 in fint(r) and
//     its last interior node in rev(t)), exactly the rule of bidi_kernel;
//   * seed rows are addressed with 64-bit begins (sbase), so graphs whose forward or
//     reverse rows pass 2^32 entries keep this plan as long as the INTERIOR rows (the ids
//     below Ni come first) fit 32-bit record begins (round-2 verdict item 6).
// Dead ends are looked up, not stored, as in bidi_kernel.  Same answers, same spill
// protocol (a spilled unit re-runs on the bidi cascade w, q, s).
constexpr int kLiteF = 128;  // ring entries per direction
// Table shape: 512 slots, 128-entry rings (9.7 KB of LDS, 16 units per CU).  Measured on
// config #2 (profiles/r03/ab_lite_shapes): a 384-slot table with 64/128-entry rings (7.4 KB,
// 21 units per CU; slots p99 230 and rings p99 35 / 72 per unit fit it) ran 0.299 vs 0.284
// ms per 10^6 requests, 512 slots with those rings 0.290: more units in flight do not pay
// for the non-power-of-two probe, and the first stage is not occupancy-bound here.
template <int H, int FF, int FB, int U = 16> struct LiteShared;

// U = 16 requests per unit: one 64-bit state word per slot, direction d's visited bits at
// 32d and pending bits at 32d + 16.  U = 32 (plan "lite32"): visited words in st (32 bits
// per direction: the meet is still one atomic) and pending words in pd.
template <int H_, int FF_, int FB_, int U_>
struct LiteShared {
    static constexpr int H = H_;             // table slots (not necessarily a power of two)
    static constexpr int HMAX = H * 7 / 8;   // load limit: a unit spills beyond it
    static constexpr int FF = FF_, FB = FB_; // ring entries, forward / backward
    static constexpr int U = U_;             // requests per unit
    static_assert(U == 16 || U == 32, "16 or 32 request bits per direction");
    using Mask = std::conditional_t<U == 16, uint16_t, uint32_t>;
    static constexpr uint32_t MASK = U == 16 ? 0xFFFFu : 0xFFFFFFFFu;
    static constexpr int psh(int d) { return U == 16 ? 32 * d + 16 : 32 * d; }  // pending bits of direction d
    alignas(16) uint32_t key[H];
    alignas(16) unsigned long long st[H];  // visited (and for U = 16 pending) bits, as above
    alignas(16) unsigned long long pd[U == 32 ? H : 2];  // U = 32: pending bits
    uint32_t ring_sd[FF + FB];             // slot | seed << 14 | degree << 16 (forward ring, then backward)
    uint32_t ring_bg[FF + FB];             // the row's first record; a seed entry: its request
    unsigned long long sbase[2][U];        // seed rows' first records (64-bit)
    unsigned long long e_beg[64];          // the chunk's entries' first records
    uint32_t c_pre[64];                    // owner map
    uint32_t c_pre2[64];                   // owner map of the prefetched forward seed rows (level 0)
    uint32_t root[U];
    Mask e_mask[64];
    __device__ __forceinline__ unsigned long long &pend(int h) {
        if constexpr (U == 32)
            return pd[h];
        else
            return st[h];
    }
    uint32_t n_used, spill, found, active;
    uint32_t head[2], tail[2];
    template <int D>
    static constexpr int ring_size() { return D ? FB : FF; }
    template <int D>
    __device__ __forceinline__ uint32_t &sd(uint32_t i) { return ring_sd[(D ? FF : 0) + i % (D ? FB : FF)]; }
    template <int D>
    __device__ __forceinline__ uint32_t &bg(uint32_t i) { return ring_bg[(D ? FF : 0) + i % (D ? FB : FF)]; }
};

using LiteShape = LiteShared<512, kLiteF, kLiteF>;
// plan core: closure rows keep tables and rings small (config #2: slots p99 116, rings p99
// 35 / 57 per unit against lite's 230 / 72), so smaller shapes fit more units per CU
using CoreShapeS = LiteShared<256, 64, 64>;
using CoreShapeM = LiteShared<256, 64, 96>;
// plan "lite32": 32 requests per unit, 1024 slots, 256-entry rings (26 KB: 6 units per CU)
using LiteShape32 = LiteShared<1024, 2 * kLiteF, 2 * kLiteF, 32>;

// find (insert == false) or find-or-insert u in a table of H slots (any H); -1 when absent
// (or the table is full)
template <int H>
__device__ __forceinline__ int lite_slot(uint32_t *key, uint32_t u, bool insert, bool &inserted) {
#ifndef KETO_LITE_PEEL
#define KETO_LITE_PEEL 0
#endif
    if constexpr ((H & (H - 1)) == 0 && !KETO_LITE_PEEL) {  // a power of two: bidi_kernel's probe
        return bidi_slot<__builtin_ctz(H)>(key, u, insert, inserted);
    } else if constexpr ((H & (H - 1)) == 0) {
        // KETO_LITE_PEEL=1: the first probe straight-line, collisions in a rolled loop —
        // fewer exec-mask instructions per push, measured slower (0.298-0.303 vs 0.284 ms
        // per 10^6 config #2 requests, profiles/r03/ab_lite_peel)
        constexpr int L = __builtin_ctz(H);
        uint32_t hh = (u * 2654435761u) >> (32 - L);
        uint32_t kv = insert ? atomicCAS(&key[hh], kEmpty, u) : key[hh];
        if (kv == kEmpty) {
            inserted = insert;
            return insert ? (int)hh : -1;
        }
        if (kv == u) return (int)hh;
#pragma unroll 1
        for (int p = 1; p < H; p++) {
            hh = (hh + 1) & (H - 1);
            kv = insert ? atomicCAS(&key[hh], kEmpty, u) : key[hh];
            if (kv == kEmpty) {
                inserted = insert;
                return insert ? (int)hh : -1;
            }
            if (kv == u) return (int)hh;
        }
        return -1;
    }
    uint32_t hh = (uint32_t)(((uint64_t)(u * 2654435761u) * (uint64_t)H) >> 32);
    for (int p = 0; p < H; p++) {
        const uint32_t kv = insert ? atomicCAS(&key[hh], kEmpty, u) : key[hh];
        if (kv == kEmpty) {
            if (!insert) return -1;
            inserted = true;
            return (int)hh;
        }
        if (kv == u) return (int)hh;
        hh = hh + 1 == (uint32_t)H ? 0u : hh + 1;
    }
    return -1;
}

struct LiteLevel {
    uint32_t lookup, sread;  // for the direction being expanded
    uint32_t head;           // the direction's ring: entries before it are read (ring_size check)
    // plan core (CL): requests whose TERMINAL pushes (closure-row entries) are lookups —
    // the other side is complete, or this level completes this side and the request
    // closes after it (lite_unit)
    uint32_t tlook = 0;
};

// plan core: record pad flags (core_index.hpp kRecTerminal / kRecClosure)
constexpr uint32_t kPadTerminal = 0x80000000u, kPadClosure = 0x40000000u;

// one lane's push of node u (record fields deg / begin / pad) in direction D.  CL (plan
// core): a TERMINAL entry (of a closure row) is visited and never pending, looked up
// under L.tlook; a pending row that is not a closure row adds its bits to nc_acc.
template <class SH, int D, bool CL = false>
__device__ __forceinline__ void lite_push(SH &S, const LiteLevel &L, bool want, uint32_t u, uint32_t deg,
                                          uint32_t begin, uint32_t m, uint32_t &or_acc, uint32_t &deg_acc,
                                          uint32_t pad = 0, uint32_t *nc_acc = nullptr) {
    const bool term = CL && (pad & kPadTerminal);
    const uint32_t lk = m & (L.lookup | (term ? L.tlook : (deg ? 0u : L.sread)));
    int h = -1;
    bool inserted = false;
    if (want) {
        const bool ins = (m & ~lk) != 0;
        h = lite_slot<SH::H>(S.key, u, ins, inserted);
        if (h < 0 && ins) S.spill = 1;
    }
    const uint64_t bal = __ballot(inserted);
    if (bal && (threadIdx.x & 63) == (unsigned)(__ffsll((unsigned long long)bal) - 1))
        atomicAdd(&S.n_used, (uint32_t)__popcll(bal));
    bool app = false;
    if (h >= 0) {
        // one 64-bit atomic: the old word carries the other direction's visited bits, so of
        // two pushes that complete a meet the later one sees it.  A push whose every bit is
        // a lookup only reads the word: lookups happen while the other direction inserts
        // nothing more for those requests, and nothing reads a lookup's own bits later
        const unsigned long long old = (m & ~lk) ? atomicOr(&S.st[h], (unsigned long long)m << (32 * D))
                                                 : __atomic_load_n(&S.st[h], __ATOMIC_RELAXED);
        uint32_t newly = m & ~(uint32_t)(old >> (32 * D)) & SH::MASK;
        const uint32_t meet = newly & (uint32_t)(old >> (32 - 32 * D)) & SH::MASK;
        if (meet) atomicOr(&S.found, meet);
        newly &= ~(meet | lk);
        if (newly && deg) {
            const unsigned long long o2 = atomicOr(&S.pend(h), (unsigned long long)newly << SH::psh(D));
            app = !((uint32_t)(o2 >> SH::psh(D)) & SH::MASK);
            or_acc |= newly;
            deg_acc += app ? deg : 0u;
            if constexpr (CL)
                if (!(pad & kPadClosure)) *nc_acc |= newly;
        }
    }
    const uint32_t idx = lds_append(app, &S.tail[D]);
    if (app) {
        if (idx - L.head < (uint32_t)SH::template ring_size<D>() && deg <= 0xFFFFu) {
            S.template sd<D>(idx) = (uint32_t)h | (deg << 16);
            S.template bg<D>(idx) = begin;
        } else {
            S.spill = 1;
        }
    }
}

// Expand this chunk's entries in direction D: lane j holds entry j's degree (0: nothing
// taken); its mask is S.e_mask[j] (SEED: bit j), its first record S.e_beg[j] (SEED: the
// seed row's, S.sbase[D][j]).  Edge-balanced: an owner map per 64-edge chunk in `own`
// (each entry writes its index at its first position, a prefix max fills the gaps), record
// loads of the next 64 edges issued before this chunk's pushes.  `pre`: chunk 0 was
// already fetched by lite_fetch0 (with the same `own`), so its loads overlapped other work.
struct LiteEdge {
    uint32_t lo, ls;
    FRec rc;
};

template <class SH, int D, bool SEED>
__device__ __forceinline__ void lite_fetch(SH &S, const FRec *rec, uint32_t *own, uint32_t my_deg, uint32_t start,
                                           uint32_t total, uint32_t eb, LiteEdge &x) {
    const uint32_t lane = threadIdx.x;
    if (my_deg && start < eb + 64 && start + my_deg > eb) own[(start > eb ? start : eb) - eb] = lane;
    __syncthreads();
    const int o = wave_incl_max_i32((int)own[lane]);
    x.lo = (uint32_t)(o < 0 ? 0 : o);
    x.ls = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(x.lo << 2), (int)start);
    const uint32_t e = min(eb + lane, total - 1);
    const unsigned long long b0 = SEED ? S.sbase[D][x.lo & (SH::U - 1)] : S.e_beg[x.lo];
    x.rc = rec[b0 + (e - x.ls)];
}

// chunk 0 of an expansion: owner map and record loads only (lite_expand with `pre` pushes it)
template <class SH, int D, bool SEED>
__device__ __forceinline__ void lite_fetch0(SH &S, const DevGraph &g, const FRec *rec, uint32_t *own,
                                            uint32_t my_deg, LiteEdge &x) {
    const uint32_t incl = wave_incl_sum_u32(my_deg);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    own[threadIdx.x] = 0xFFFFFFFFu;
    if (total) lite_fetch<SH, D, SEED>(S, rec - g.seed_shift, own, my_deg, incl - my_deg, total, 0, x);
}

template <class SH, int D, bool SEED = false, bool CL = false>
__device__ __forceinline__ void lite_expand(SH &S, const DevGraph &g, const FRec *rec, const LiteLevel &L,
                                            uint32_t my_deg, uint64_t &edges, uint32_t &or_acc, uint32_t &deg_acc,
                                            uint32_t *own, const LiteEdge *pre = nullptr, uint32_t *nc_acc = nullptr) {
    const uint32_t lane = threadIdx.x;
    const uint32_t incl = wave_incl_sum_u32(my_deg);
    const uint32_t start = incl - my_deg;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (!total) return;
    rec -= g.seed_shift;  // begins carry the shift (0 outside the test knob)
    auto push = [&](uint32_t eb, const LiteEdge &x) {
        const uint32_t found = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.found);
        edges += min(64u, total - eb);  // the wave's count (uniform: scalar), not one per lane
        uint32_t m = 0;
        if (eb + lane < total) {
            m = (SEED ? (1u << (x.lo & (SH::U - 1))) : (uint32_t)S.e_mask[x.lo]) & ~found;
            if (D == 1 && x.rc.node >= g.Ni) {  // a source entry of rev(t): it can only meet r itself
                uint32_t hit = 0;
                for (uint32_t b = m; b; b &= b - 1)
                    if (S.root[__ffs(b) - 1] == x.rc.node) hit |= b & (~b + 1);
                if (hit) atomicOr(&S.found, hit);
                m = 0;
            }
        }
        lite_push<SH, D, CL>(S, L, m != 0, x.rc.node, x.rc.deg, x.rc.begin, m, or_acc, deg_acc, x.rc.pad, nc_acc);
    };
    LiteEdge a{}, b{};
    if (pre) {
        a = *pre;
    } else {
        own[lane] = 0xFFFFFFFFu;
        lite_fetch<SH, D, SEED>(S, rec, own, my_deg, start, total, 0, a);
    }
    if (total <= 64) {  // one chunk (the common level): no pipelining to pay for
        push(0, a);
        return;
    }
    for (uint32_t eb = 0;;) {
        lite_fetch<SH, D, SEED>(S, rec, own, my_deg, start, total, eb + 64, b);
        push(eb, a);
        eb += 64;
        if (eb + 64 >= total) {
            push(eb, b);
            break;
        }
        lite_fetch<SH, D, SEED>(S, rec, own, my_deg, start, total, eb + 64, a);
        push(eb, b);
        eb += 64;
        if (eb + 64 >= total) {
            push(eb, a);
            break;
        }
    }
}

// consume direction D's ring (every pending row: one atomic reads and clears its pending
// bits of D) and expand it
template <class SH, int D, bool CL = false>
__device__ __forceinline__ void lite_level(SH &S, const DevGraph &g, const FRec *rec, LiteLevel L, uint32_t open,
                                           uint64_t &edges, uint32_t &or_acc, uint32_t &deg_acc,
                                           uint32_t *nc_acc = nullptr) {
    const uint32_t lane = threadIdx.x;
    const uint32_t h0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.head[D]);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.tail[D]);
    for (uint32_t c = h0; c < t0; c += 64) {
        const uint32_t i = c + lane;
        uint32_t deg = 0, take = 0;
        if (i < t0) {
            const uint32_t w = S.template sd<D>(i), bg = S.template bg<D>(i);
            const uint32_t s = w & 0x3FFFu;
            const unsigned long long old = atomicAnd(&S.pend(s), ~((unsigned long long)SH::MASK << SH::psh(D)));
            take = (uint32_t)(old >> SH::psh(D)) & open;
            deg = take ? w >> 16 : 0u;
            // a seed row's begin is 64-bit (sbase); an interior row's is the record's 32 bits,
            // shifted like sbase by the test knob (rec is taken back by it)
            S.e_beg[lane] = (w >> 14) & 1u ? S.sbase[D][bg & (SH::U - 1)] : (unsigned long long)bg + g.seed_shift;
        }
        S.e_mask[lane] = (typename SH::Mask)take;
        L.head = min(c + 64, t0);  // these entries are read: their ring slots are free
        if (lane == 0) S.head[D] = L.head;
        __syncthreads();
        lite_expand<SH, D, false, CL>(S, g, rec, L, deg, edges, or_acc, deg_acc, S.c_pre, nullptr, nc_acc);
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t wave_or_all(uint32_t x) {
#pragma unroll
    for (int s = 32; s; s >>= 1) x |= (uint32_t)__shfl_xor((int)x, s, 64);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint32_t wave_sum_all(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum_u32(x), 63);
}

// one 16-request unit by one wave (seed as bidi_load_rows loads it on lanes < 16).
// CL (plan core, core_index.hpp): records may name CLOSURE rows.  Per direction the unit
// tracks the requests with a pending row that is not a closure row (nc); while every
// request pending on a side has only closure rows pending there, that side alone is
// expanded next and completes in that level, so its terminal entries are lookups for
// the requests that close after it (the other side's seed row read).
template <class SH, bool CL = false>
__device__ __forceinline__ void lite_unit(SH &S, const DevGraph &g, const FRec *frec, const FRec *brec,
                                          const BidiSeed &seed, uint64_t *allowed, const uint64_t unit,
                                          uint32_t *spill_out, unsigned int *spill_count, unsigned long long *stats,
                                          unsigned long long *stamp = nullptr, uint32_t ridx = KETOGPU_NODE_NONE,
                                          bool gathered = false) {
    const uint32_t lane = threadIdx.x;
    // gathered (plan label's second stage): the unit's requests are scattered over the
    // batch, lane j < U holding request j's index (ridx; NONE: no request); results and
    // spills go per request instead of per unit
    auto spill_unit = [&]() {
        if (!gathered) {
            if (lane == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        } else {
            const bool w = lane < SH::U && ridx != KETOGPU_NODE_NONE;
            const uint32_t at = lds_append(w, spill_count);
            if (w) spill_out[at] = ridx;
        }
    };
    if (stamp) stamp[0] = __builtin_amdgcn_s_memtime();
    const uint64_t c0 = unit * SH::U;
    for (int i = lane; i < SH::H / 4; i += 64) reinterpret_cast<uint4 *>(S.key)[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    for (int i = lane; i < SH::H / 2; i += 64) reinterpret_cast<uint4 *>(S.st)[i] = make_uint4(0, 0, 0, 0);
    if constexpr (SH::U == 32)
        for (int i = lane; i < SH::H / 2; i += 64) reinterpret_cast<uint4 *>(S.pd)[i] = make_uint4(0, 0, 0, 0);
    if (lane == 0) S.n_used = S.spill = S.found = S.active = S.head[0] = S.head[1] = S.tail[0] = S.tail[1] = 0;
    const uint32_t r = seed.r, t = seed.t;
    uint64_t rows = 0, edges = 0;
    if (lane < SH::U) {
        if (r != KETOGPU_NODE_NONE && r < kDynBase) {
            rows += 2;
            // nothing reaches a t without predecessors (!=: the two-tier mode's begins are
            // offsets from another array and may wrap, tier.hpp)
            if (seed.re != seed.rb) atomicOr(&S.active, 1u << lane);
        }
        if (r != KETOGPU_NODE_NONE && r >= kDynBase) S.spill = 1;
        S.root[lane] = r;
        S.sbase[0][lane] = seed.fb + g.seed_shift;
        S.sbase[1][lane] = seed.rb + g.seed_shift;
    }
    __syncthreads();
    if (S.spill) {
        spill_unit();
        return;
    }
    uint32_t active = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.active);
    // seeds: r forward-visited and t backward-visited at distance 0 (t = r excluded: a meet
    // needs >= 1 edge); both rows short: both read at level 0, else both become pending
    const bool v = lane < SH::U && ((active >> lane) & 1u);
    const uint32_t bit = 1u << (lane & (SH::U - 1));
    const uint32_t rdeg = (uint32_t)(seed.fe - seed.fb), tdeg = (uint32_t)(seed.re - seed.rb);
    const bool eager = rdeg <= g.seed_max && tdeg <= g.seed_max;
    uint32_t pend_mask[2];
    for (int side = 0; side < 2; side++) {
        const uint32_t u = side ? t : r, deg = side ? tdeg : rdeg;
        bool inserted = false;
        const int h = v ? lite_slot<SH::H>(S.key, u, true, inserted) : -1;
        const uint64_t bal = __ballot(inserted);
        if (lane == 0) S.n_used += (uint32_t)__popcll(bal);
        const bool pend = h >= 0 && !eager && deg;
        bool app = false;
        if (h >= 0) {
            const unsigned long long vb = (side == 0 || t != r) ? (unsigned long long)bit << (32 * side) : 0ull;
            const unsigned long long pb = pend ? (unsigned long long)bit << SH::psh(side) : 0ull;
            unsigned long long oldp;
            if constexpr (SH::U == 16) {
                oldp = atomicOr(&S.st[h], vb | pb);
            } else {
                if (vb) atomicOr(&S.st[h], vb);
                oldp = pb ? atomicOr(&S.pd[h], pb) : 0ull;
            }
            app = pend && !((uint32_t)(oldp >> SH::psh(side)) & SH::MASK);
        }
        pend_mask[side] = (uint32_t)__ballot(pend);
        const uint32_t idx = lds_append(app, &S.tail[side]);  // idx < 16 <= F
        if (app) {  // idx < 16 <= every ring's size
            if (deg > 0xFFFFu) S.spill = 1;
            if (side) {
                S.template sd<1>(idx) = (uint32_t)h | (1u << 14) | (deg << 16);
                S.template bg<1>(idx) = lane;
            } else {
                S.template sd<0>(idx) = (uint32_t)h | (1u << 14) | (deg << 16);
                S.template bg<0>(idx) = lane;
            }
        }
    }
    uint32_t rpend = pend_mask[0], tpend = pend_mask[1];  // seed rows not read yet
    // pending-row presence and degree totals per direction
    uint32_t pf = rpend, pb = tpend, sf = 0, sb = 0;
    uint32_t acc_or[2] = {0, 0}, acc_deg[2] = {0, 0};
    // CL: requests with a pending row that is not a closure row, per direction (a pending
    // seed row is a one-hop row)
    uint32_t nc_f = rpend, nc_b = tpend, nc_acc[2] = {0, 0};
    for (int side = 0; side < 2; side++) {  // the pending seed rows' degrees
        const uint32_t d = (lane < SH::U && ((pend_mask[side] >> lane) & 1u)) ? (side ? tdeg : rdeg) : 0u;
        (side ? sb : sf) = wave_sum_all(d);
    }
    if (stamp) stamp[1] = __builtin_amdgcn_s_memtime();
    // level 0: the eager seed rows.  rev(t) first (every push inserts), then fint(r): by
    // then t's row is complete, so a forward dead end (a group with no interior successor:
    // most of a document's grants) can only meet t or an entry of rev(t) and is looked up,
    // not stored
    {
        const bool e = v && eager;
        const uint32_t eager_mask = (uint32_t)__ballot(e) & SH::MASK;
        const uint32_t df = (lane < SH::U && e) ? rdeg : 0u, db = (lane < SH::U && e) ? tdeg : 0u;
        // the forward rows' first 64 records are loaded before the backward pushes, so
        // the two dependent expansions of level 0 wait for HBM once
        LiteEdge f0{};
        lite_fetch0<SH, 0, true>(S, g, frec, S.c_pre2, df, f0);
        lite_expand<SH, 1, true, CL>(S, g, brec, LiteLevel{0, 0, 0}, db, edges, acc_or[1], acc_deg[1], S.c_pre,
                                     nullptr, &nc_acc[1]);
        __syncthreads();
        lite_expand<SH, 0, true, CL>(S, g, frec, LiteLevel{0, eager_mask, 0}, df, edges, acc_or[0], acc_deg[0],
                                     S.c_pre2, &f0, &nc_acc[0]);
        __syncthreads();
        pf |= wave_or_all(acc_or[0]);
        pb |= wave_or_all(acc_or[1]);
        sf += wave_sum_all(acc_deg[0]);
        sb += wave_sum_all(acc_deg[1]);
        if constexpr (CL) {
            nc_f |= wave_or_all(nc_acc[0]);
            nc_b |= wave_or_all(nc_acc[1]);
        }
    }
    if (stamp) stamp[2] = __builtin_amdgcn_s_memtime();
    bool spilled = false;
    uint32_t n_levels = 0, ring_max[2] = {0, 0};
    for (;;) {
        __syncthreads();
        const uint32_t found = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.found);
        uint32_t open = active & ~found;
        if (stamp)
            for (int d = 0; d < 2; d++) ring_max[d] = max(ring_max[d], S.tail[d] - S.head[d]);
        if (S.spill || (S.n_used > (uint32_t)SH::HMAX && open)) {  // undecided requests, table over its load
            spilled = true;
            break;
        }
        const uint32_t fc = open & ~pf, bc = open & ~pb;
        const uint32_t closed = (fc & ~tpend) | (bc & ~rpend) | (fc & bc);
        active &= ~closed;
        open &= ~closed;
        if (!open) break;
        const bool want_f = (pf & open) != 0, want_b = (pb & open) != 0;
        // CL: a side whose open pending requests have only closure rows pending completes
        // when expanded alone
        const bool cf = CL && want_f && !(nc_f & open & pf), cb = CL && want_b && !(nc_b & open & pb);
        bool do_f, do_b;
        if (cf || cb) {
            do_b = cb && (!cf || sb <= sf);
            do_f = !do_b;
        } else if (want_f && want_b && sf <= g.both_max && sb <= g.both_max) {
            do_f = do_b = true;
        } else if (want_f && want_b) {
            do_f = sf <= sb;
            do_b = !do_f;
        } else {
            do_f = want_f;
            do_b = want_b;
        }
        // bits of requests whose OTHER side is closed: only looked up (a meet or nothing);
        // a dead end (no row in this direction) is only looked up once the other side's
        // seed row was read in an earlier level (it can meet nothing else).  CL: terminal
        // entries also of requests this level completes and closes (the side expanded
        // alone, only closure rows pending on it, the other side's seed row read): the
        // other side inserts nothing more for them
        n_levels++;
        if (do_f) {
            const uint32_t tl = CL && !do_b ? open & ~nc_f & ~tpend : 0u;
            const LiteLevel L{open & bc, ~tpend, 0, (open & bc) | tl};
            acc_or[0] = acc_deg[0] = nc_acc[0] = 0;
            lite_level<SH, 0, CL>(S, g, frec, L, open, edges, acc_or[0], acc_deg[0], &nc_acc[0]);
        }
        if (do_b) {
            const uint32_t tl = CL && !do_f ? open & ~nc_b & ~rpend : 0u;
            const LiteLevel L{open & fc, ~rpend, 0, (open & fc) | tl};
            acc_or[1] = acc_deg[1] = nc_acc[1] = 0;
            lite_level<SH, 1, CL>(S, g, brec, L, open, edges, acc_or[1], acc_deg[1], &nc_acc[1]);
        }
        if (do_f) {
            pf = wave_or_all(acc_or[0]);
            sf = wave_sum_all(acc_deg[0]);
            if constexpr (CL) nc_f = wave_or_all(nc_acc[0]);
            rpend = 0;
        }
        if (do_b) {
            pb = wave_or_all(acc_or[1]);
            sb = wave_sum_all(acc_deg[1]);
            if constexpr (CL) nc_b = wave_or_all(nc_acc[1]);
            tpend = 0;
        }
    }
    __syncthreads();
    if (spilled || S.spill) {
        spill_unit();
        return;
    }
    if (stamp) {  // KETOGPU_STAMPS=1: phase cycles, levels and table load per unit (report_stamps)
        stamp[3] = stamp[4] = __builtin_amdgcn_s_memtime();
        stamp[5] = n_levels;
        stamp[6] = S.n_used;
        stamp[7] = 1;
        stamp[12] = ring_max[0];
        stamp[13] = ring_max[1];
    }
#pragma unroll
    for (int s = 32; s; s >>= 1) rows += __shfl_down(rows, s, 64);  // edges: already the wave's
    if (lane == 0) {
        const uint32_t res = S.found & SH::MASK;
        if (res && !gathered) atomicOr((unsigned long long *)&allowed[c0 >> 6], (unsigned long long)res << (c0 & 63));
        atomicAdd(&stat_slot(stats)[0], (unsigned long long)rows);
        atomicAdd(&stat_slot(stats)[1], (unsigned long long)edges);
    }
    if (gathered && lane < SH::U && ridx != KETOGPU_NODE_NONE && ((S.found >> lane) & 1u))
        atomicOr((unsigned long long *)&allowed[ridx >> 6], 1ull << (ridx & 63));
}

// plan "lite" first stage over HBM-resident requests (unit0: a chunk's first unit); CL:
// plan "core" (record arrays with closure rows, core_index.hpp)
template <class SH, bool CL = false>
__global__ __launch_bounds__(64) void lite_kernel(DevGraph g, const FRec *frec, const FRec *brec, const uint32_t *roots,
                                                  const uint32_t *targets, uint64_t n, uint64_t *allowed,
                                                  uint32_t *spill_out, unsigned int *spill_count,
                                                  unsigned long long *stats, uint64_t unit0,
                                                  unsigned long long *stamps) {
    __shared__ SH S;
    const uint64_t units = (n + SH::U - 1) / SH::U;
    const uint64_t unit = unit0 + blockIdx.x;
    uint32_t r, t;
    bidi_load_rt<SH::U>(unit, units, roots, targets, n, r, t);
    unsigned long long *stamp =
        (stamps && blockIdx.x < 65536 && threadIdx.x == 0) ? stamps + (size_t)blockIdx.x * 16 : nullptr;
    lite_unit<SH, CL>(S, g, frec, brec, CL ? core_load_rows(g, frec, brec, r, t) : bidi_load_rows(g, r, t), allowed,
                      unit, spill_out, spill_count, stats, stamp);
}

// plan "lite" first stage over pinned host requests read in place (bidi_host_kernel's
// prologue: K units per workgroup, requests validated and stored in HBM for the spill stages)
template <int K, class SH, bool CL = false>
__global__ __launch_bounds__(64) void lite_host_kernel(DevGraph g, const FRec *frec, const FRec *brec,
                                                       const uint32_t *hr, const uint32_t *ht, uint32_t *dr,
                                                       uint32_t *dt, uint64_t n, uint64_t *allowed, uint32_t *spill_out,
                                                       unsigned int *spill_count, unsigned long long *stats,
                                                       unsigned long long *first_bad) {
    __shared__ SH S;
    uint32_t r[K], t[K];
    if constexpr (SH::U == 16) {
        host_unit_requests<K>(g, hr, ht, dr, dt, n, first_bad, r, t);
    } else {  // 32-request units (plan lite32, an A/B plan): lanes < 32 read their own
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t c = ((uint64_t)blockIdx.x * K + k) * SH::U + threadIdx.x;
            r[k] = t[k] = KETOGPU_NODE_NONE;
            if (threadIdx.x < SH::U && c < n) {
                r[k] = hr[c];
                t[k] = ht[c];
                if ((r[k] != KETOGPU_NODE_NONE && r[k] >= g.Nx) || (t[k] != KETOGPU_NODE_NONE && t[k] >= g.N)) {
                    atomicMin(first_bad, (unsigned long long)c);
                    r[k] = t[k] = KETOGPU_NODE_NONE;
                }
                dr[c] = r[k];
                dt[c] = t[k];
            }
        }
    }
    const uint64_t units = (n + SH::U - 1) / SH::U;
#pragma unroll 1
    for (int k = 0; k < K; k++) {
        const uint64_t unit = (uint64_t)blockIdx.x * K + k;
        if (unit >= units) break;
        uint32_t rk = r[0], tk = t[0];
#pragma unroll
        for (int j = 1; j < K; j++)
            if (j == k) rk = r[j], tk = t[j];
        lite_unit<SH, CL>(S, g, frec, brec, CL ? core_load_rows(g, frec, brec, rk, tk) : bidi_load_rows(g, rk, tk),
                          allowed, unit, spill_out, spill_count, stats);
        __syncthreads();
    }
}

// ----------------------------------------------------------------------- plan label
// 2-hop reachability labels (labels.hpp): per request one S list (target t) and one P list
// (root r), each behind a fixed-size HEAD of HS / HP words [count | overflow start / 16 |
// mask lo | mask hi | entries ascending | 0xFFFFFFFF pad]; allowed <=> the masks share a
// bit, the lists share a landmark, or r (not interior) is among S's raw entries (the
// one-edge test).  One wave per 16-request unit: four lanes per request read its two heads
// (one dependent HBM read each, both in flight at once), and the shorter inline landmark
// list is looked up in the other by a branchless binary search in LDS.  A request the heads
// cannot settle (labels.hpp: the prefix rules) goes to the dense pass over the overflow
// lists.  A request without labels (a wildcard root, or the KETOGPU_LABEL_REST_PERMILLE test
// knob) is listed (one request index each) for the second stage, label_rest_kernel: plan
// lite's traversal over the listed requests, gathered 16 to a unit.
struct LabelGraph {
    const uint32_t *P, *S;  // head arrays (+ overflow lists)
    uint32_t ni;            // interior nodes: landmark ranks are below, raw entries and non-interior roots not
};
// The unlabelled requests' list is sharded: unit u appends to region u % kRestShards of
// the list (region capacity `rest_cap` = 16 x ceil(units / kRestShards)) at counter
// rest_count[(u % kRestShards) * kRestStride] — one cache line per counter, so appends do
// not serialize on one address.  Two counter sets alternate between calls: a call's first
// stage (workgroup 0) clears the other set for the next call.
constexpr int kRestShards = 64, kRestStride = 32;
struct LabelRest {
    uint32_t *list;                    // request indices (the rest list)
    unsigned int *count, *next_count;  // this call's counters, the next call's (cleared here)
    uint64_t cap;                      // entries per region
    uint4 *rec = nullptr;              // the full list: two records per request, {request, root, target,
                                       // |S|} and {|P|, S overflow start / 16, P overflow start / 16, 0}
};
// A request's two heads in LDS, as read (word k of the head at position k; the entries
// from word 4), rows of HS + 4 / HP + 4 words: 16-byte aligned, and the 16 requests' rows
// start in different banks
template <int HS, int HP>
struct alignas(16) LabelShared {
    uint32_t S[16 * (HS + 4)], P[16 * (HP + 4)];
};

// x among the n ascending entries of a list (LDS or global memory)
__device__ __forceinline__ bool label_find_n(const uint32_t *S, uint32_t n, uint32_t x) {
    const uint32_t n0 = n;
    uint32_t lo = 0;
    while (n) {
        const uint32_t half = n >> 1;
        if (S[lo + half] < x) {
            lo += half + 1;
            n -= half + 1;
        } else {
            n = half;
        }
    }
    return lo < n0 && S[lo] == x;
}

// this lane's W words of a head (lane `sub` of the request's four: words [W sub, W sub + W))
template <int W>
__device__ __forceinline__ void label_head_load(const uint32_t *head, uint32_t sub, uint32_t (&w)[W]) {
    if constexpr (W == 2) {
        const uint2 a = reinterpret_cast<const uint2 *>(head)[sub];
        w[0] = a.x, w[1] = a.y;
    } else {
#pragma unroll
        for (int k = 0; k < W / 4; k++) {
            const uint4 a = reinterpret_cast<const uint4 *>(head)[(W / 4) * sub + k];
            w[4 * k] = a.x, w[4 * k + 1] = a.y, w[4 * k + 2] = a.z, w[4 * k + 3] = a.w;
        }
    }
}
// word J (< 4: count, overflow start, mask lo, mask hi) of the request's head on all four of
// its lanes: a DPP quad broadcast (the four lanes of a request are one DPP quad)
template <int W, int J>
__device__ __forceinline__ uint32_t label_word(const uint32_t (&w)[W]) {
    constexpr int src = J / W;
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w[J % W], src * 0x55, 0xf, 0xf, false);  // quad_perm [src x 4]
}
// the head image to LDS (aligned rows)
template <int W>
__device__ __forceinline__ void label_to_lds(uint32_t *L, const uint32_t (&w)[W], uint32_t sub) {
    if constexpr (W == 2) {
        reinterpret_cast<uint2 *>(L)[sub] = make_uint2(w[0], w[1]);
    } else {
#pragma unroll
        for (int k = 0; k < W / 4; k++)
            reinterpret_cast<uint4 *>(L)[(W / 4) * sub + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    }
}
// entries below x among the first E ascending entries at L (LDS; positions past the list
// hold 0xFFFFFFFF or larger entries): a branchless binary search (E = head - 4, up to 60)
template <int E>
__device__ __forceinline__ uint32_t label_lower_e(const uint32_t *L, uint32_t x) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
        if (step <= (uint32_t)E && pos + step <= (uint32_t)E && L[pos + step - 1] < x) pos += step;
    return pos;
}
// x among the first E entries at L
template <int E>
__device__ __forceinline__ bool label_find_e(const uint32_t *L, uint32_t x) {
    const uint32_t pos = label_lower_e<E>(L, x);
    return pos < (uint32_t)E && L[pos] == x;
}

// x among the first E ascending entries at L (LDS, 16-byte aligned) in two dependent LDS
// rounds: the last entries of the 8-entry blocks (independent reads) give x's block, whose 8
// entries are then read at once (two 16-byte reads) — against the binary search's chain of
// log2(E) dependent reads.  Words at positions >= E are never compared (the image row's
// words past the head are not written).  lower: the entries below x instead
template <int E, bool LOWER>
__device__ __forceinline__ uint32_t label_block8(const uint32_t *L, uint32_t x) {
    constexpr int NB = (E + 7) / 8;
    uint32_t blk = 0;
#pragma unroll
    for (int b = 0; b + 1 < NB; b++) blk += L[8 * b + 7] < x;
    const uint4 u = *reinterpret_cast<const uint4 *>(L + 8 * blk), v = *reinterpret_cast<const uint4 *>(L + 8 * blk + 4);
    const uint32_t w[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    uint32_t r = LOWER ? 8 * blk : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const bool in = 8 * blk + i < (uint32_t)E;
        if (LOWER)
            r += in && w[i] < x;
        else
            r |= in && w[i] == x;
    }
    return r;
}

// x in the head image `row` (LDS) among its first E entries (H: the head's words)
template <int E, int H, bool LOWER>
__device__ __forceinline__ uint32_t label_lookup(const uint32_t *row, uint32_t x) {
    return label_block8<E, LOWER>(row + kHeadFixed, x);
}

// KETO_LABEL_MEET: how the shorter inline landmark list meets the other head.  0 (default):
// the shorter list's entries round-robin over the request's four lanes, each looked up in the
// other list in LDS by label_block8 (two dependent LDS rounds); 2: the same by a binary search
// (log2(E) dependent rounds: config #3's long lists pay for it).  Measured and dropped: every
// lane reading the shorter list's entries and comparing them with its quarter of the other
// head in registers (2.8x slower at 64-word heads, profiles/r06/ab).  Four lookups per lane in flight
// at once instead of one at a time: no faster (config #3 shape), 10% slower (config #2); the
// block splitters stored as a row of their own (two 16-byte reads instead of one word per
// block): 8% slower on the config #3 shape, equal on config #2; padded rows instead of the
// per-entry bounds test in label_block8 (fewer VALU instructions): 5-8% slower
// (profiles/r06/ab/ab_*_pad.jsonl); a 64-word head's second line read only when its list
// needs it (both heads' first lines together, then the second lines): equal traffic to the
// kernel's bound, 5% slower (ab_f_lines2 / ab_f_whole2)
#ifndef KETO_LABEL_MEET
#define KETO_LABEL_MEET 0
#endif

// A unit of 16 requests by one wave (four lanes per request), the heads' inline entries
// only: a request the heads do not settle is listed in F for the dense second pass
// (label_full_kernel), so no wave waits on one request's second read.
template <int HS, int HP>
__device__ __forceinline__ void label_unit(LabelShared<HS, HP> &sh, const LabelGraph &L, uint32_t r_lane,
                                           uint32_t t_lane, uint64_t *allowed, const uint64_t unit,
                                           const LabelRest &R, const LabelRest &F, unsigned long long *stats) {
    static_assert((HS == 8 || HS == 16 || HS == 32 || HS == 64) && (HP == 8 || HP == 16 || HP == 32 || HP == 64),
                  "heads of 8, 16, 32 or 64 words");
    constexpr int SW = HS / 4, PW = HP / 4;                                   // head words per lane
    constexpr uint32_t CS = HS - kHeadFixed, CP = HP - kHeadFixed;            // inline entries
    const uint32_t lane = threadIdx.x & 63, q = lane >> 2, sub = lane & 3;
    const uint32_t r = (uint32_t)__shfl((int)r_lane, (int)q, 64), t = (uint32_t)__shfl((int)t_lane, (int)q, 64);
    const bool some = r != KETOGPU_NODE_NONE && t != KETOGPU_NODE_NONE;
    const bool valid = some && r < kDynBase;
    uint32_t sw[SW], pw[PW];
#pragma unroll
    for (int k = 0; k < SW; k++) sw[k] = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < PW; k++) pw[k] = 0xFFFFFFFFu;
    if (valid) {  // both heads in flight at once: one dependent HBM read per request
        label_head_load<SW>(L.S + (uint64_t)t * HS, sub, sw);
        label_head_load<PW>(L.P + (uint64_t)r * HP, sub, pw);
    }
    const uint32_t ns = label_word<SW, 0>(sw), np = label_word<PW, 0>(pw);
    const bool labelled = valid && ns != kNoLabel && np != kNoLabel;
    const uint64_t smask = (uint64_t)label_word<SW, 2>(sw) | (uint64_t)label_word<SW, 3>(sw) << 32;
    const uint64_t pmask = (uint64_t)label_word<PW, 2>(pw) | (uint64_t)label_word<PW, 3>(pw) << 32;
    uint32_t *Sl = sh.S + q * (HS + 4), *Pl = sh.P + q * (HP + 4);
    label_to_lds<SW>(Sl, sw, sub);
    label_to_lds<PW>(Pl, pw, sub);
    const uint32_t *Se = Sl + kHeadFixed, *Pe = Pl + kHeadFixed;  // the inline entries
    const uint32_t shard = (uint32_t)(unit % kRestShards);
    // a request without labels (or with a wildcard root): listed for the second stage
    {
        const bool rest = sub == 0 && some && !labelled;
        const uint32_t at = lds_append(rest, R.count + shard * kRestStride);
        if (rest) R.list[shard * R.cap + at] = (uint32_t)(unit * 16 + q);
    }
    wave_sync();  // (the images: this wave's own rows)
    bool hit = labelled && (smask & pmask) != 0;
    // S's inline landmarks: its inline entries below Ni (the raw entries follow them)
    const uint32_t es = !labelled ? 0u : KETO_LABEL_MEET == 2 ? label_lower_e<CS>(Se, L.ni) : label_lookup<CS, HS, true>(Sl, L.ni);
    const uint32_t ep = min(np, CP);
    // 1. the inline landmark prefixes: the shorter walked, round-robin over the request's
    //    four lanes, each entry searched in the other; the one-edge test (a non-interior root
    //    among S's inline raw entries) on the fourth lane
    if (labelled && !hit) {
        if (KETO_LABEL_MEET == 2) {
            if (es <= ep)
                for (uint32_t k = sub; k < es && !hit; k += 4) hit = label_find_e<CP>(Pe, Se[k]);
            else
                for (uint32_t k = sub; k < ep && !hit; k += 4) hit = label_find_e<CS>(Se, Pe[k]);
            if (sub == 3 && !hit && r >= L.ni) hit = label_find_e<CS>(Se, r);
        } else {
            if (es <= ep)
                for (uint32_t k = sub; k < es && !hit; k += 4) hit = label_lookup<CP, HP, false>(Pl, Se[k]);
            else
                for (uint32_t k = sub; k < ep && !hit; k += 4) hit = label_lookup<CS, HS, false>(Sl, Pe[k]);
            if (sub == 3 && !hit && r >= L.ni) hit = label_lookup<CS, HS, false>(Sl, r);
        }
    }
    // 2. a request neither hit nor settled by its heads (labels.hpp): listed for
    //    label_full_kernel, with both counts and overflow starts (the dense pass then needs no
    //    head again).  Settled: no landmark can be missing from the prefixes — S's landmarks
    //    whole (its list inline, or its last inline entry raw) and P's whole, or one whole with
    //    its largest landmark <= the other's last inline one — and the raw test settled: r
    //    interior, S whole inline, or r <= S's last inline entry
    {
        const uint64_t hb = __ballot(hit);
        const uint32_t os = label_word<SW, 1>(sw), op = label_word<PW, 1>(pw);
        bool full = false;
        if (sub == 0 && labelled && !((hb >> lane) & 0xF)) {
            const uint32_t s_end = Se[CS - 1];  // (ns > CS: the last inline entry)
            const bool s_whole = ns <= CS || s_end >= L.ni, p_whole = np <= CP;
            const uint32_t s_last = es ? Se[es - 1] : 0u, p_last = ep ? Pe[ep - 1] : 0u;
            const bool lm_done = es == 0 || np == 0 || (s_whole && (p_whole || s_last <= p_last)) ||
                                 (p_whole && p_last <= s_last);
            const bool raw_done = r < L.ni || ns <= CS || r <= s_end;
            full = !(lm_done && raw_done);
        }
        const uint32_t at = lds_append(full, F.count + shard * kRestStride);
        if (full) {
            uint4 *rec = F.rec + 2 * (shard * F.cap + at);
            rec[0] = make_uint4((uint32_t)(unit * 16 + q), r, t, ns);
            rec[1] = make_uint4(np, os, op, 0u);
        }
    }
    const uint64_t bits = __ballot(hit);
    // statistics: 2 rows (heads) and the entries read (both lists and the masks) per request
    const uint32_t rows = wave_sum_all(labelled && sub == 0 ? 2u : 0u);
    const uint32_t ent = wave_sum_all(labelled && sub == 0 ? ns + np + kHeadFixed : 0u);
    // bit j of the unit's result = any of the request's four lanes (scalar bit compression)
    uint64_t x = bits | bits >> 1;
    x = (x | x >> 2) & 0x1111111111111111ull;
    x = (x | x >> 3) & 0x0303030303030303ull;
    x = (x | x >> 6) & 0x000F000F000F000Full;
    x = (x | x >> 12) & 0x000000FF000000FFull;
    x = (x | x >> 24) & 0xFFFFull;
    if (lane == 0) {
        // the unit's 16 result bits are the 16-bit word `unit` of the result array: a plain
        // store (every unit writes its own, zeros included), so the array needs no clearing
        // before the first stage; the later passes OR their bits in after it
        reinterpret_cast<uint16_t *>(allowed)[unit] = (uint16_t)x;
        if (stats) {  // (lean calls: none)
            atomicAdd(&stat_slot(stats)[0], (unsigned long long)rows);
            atomicAdd(&stat_slot(stats)[2], (unsigned long long)ent);  // u32 entries: 4 B each
        }
    }
}

// the next call's list counters (rest and full), cleared by wave 0 of workgroup 0
__device__ __forceinline__ void label_clear_next(const LabelRest &R, const LabelRest &F) {
    if (blockIdx.x == 0 && threadIdx.x < 64) {  // 64 lanes: every shard
        R.next_count[threadIdx.x * kRestStride] = 0u;
        F.next_count[threadIdx.x * kRestStride] = 0u;
    }
}

template <int HS, int HP>
__global__ __launch_bounds__(64) void label_kernel(LabelGraph L, const uint32_t *roots, const uint32_t *targets,
                                                   uint64_t n, uint64_t *allowed, LabelRest R, LabelRest F,
                                                   unsigned long long *stats, uint64_t unit0) {
    __shared__ LabelShared<HS, HP> sh;
    if (unit0 == 0) label_clear_next(R, F);
    const uint64_t units = (n + 15) / 16;
    const uint64_t unit = unit0 + blockIdx.x;
    uint32_t r, t;
    bidi_load_rt<16>(unit, units, roots, targets, n, r, t);
    label_unit<HS, HP>(sh, L, r, t, allowed, unit, R, F, stats);
    // the last result word's 16-bit parts past the last unit (no unit writes them)
    if (unit + 1 == units && threadIdx.x == 0)
        for (uint64_t u = units; u < (units + 3) / 4 * 4; u++) reinterpret_cast<uint16_t *>(allowed)[u] = 0;
}

// pinned host requests read in place: four waves per workgroup, one unit each; wave 0 reads
// the four units' requests (host_unit_requests: two 256-byte PCIe reads) and hands them over
// in LDS, so the units' head reads and searches run side by side
template <int HS, int HP>
__global__ __launch_bounds__(256) void label_host_kernel(DevGraph g, LabelGraph L, const uint32_t *hr,
                                                         const uint32_t *ht, uint32_t *dr, uint32_t *dt, uint64_t n,
                                                         uint64_t *allowed, LabelRest R, LabelRest F,
                                                         unsigned long long *stats, unsigned long long *first_bad) {
    __shared__ LabelShared<HS, HP> sh[4];
    __shared__ uint32_t rq[2][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    label_clear_next(R, F);
    if (wave == 0) {
        uint32_t r[4], t[4];
        host_unit_requests<4>(g, hr, ht, dr, dt, n, first_bad, r, t);
        if (lane < 16)
#pragma unroll
            for (int k = 0; k < 4; k++) rq[0][16 * k + lane] = r[k], rq[1][16 * k + lane] = t[k];
    }
    __syncthreads();
    const uint64_t units = (n + 15) / 16;
    const uint64_t unit = (uint64_t)blockIdx.x * 4 + wave;
    if (unit >= units) return;  // (a whole wave: no barrier follows)
    const uint32_t rk = lane < 16 ? rq[0][16 * wave + lane] : KETOGPU_NODE_NONE;
    const uint32_t tk = lane < 16 ? rq[1][16 * wave + lane] : KETOGPU_NODE_NONE;
    label_unit<HS, HP>(sh[wave], L, rk, tk, allowed, unit, R, F, stats);
}

// The dense second pass over the requests the first stage's heads did not settle (F: two
// records per request carrying both counts and overflow starts): gathered 16 to a wave,
// four lanes per request, persistent.  It answers from the whole lists: the landmark
// intersection (S's raw entries never meet P's landmarks) and the one-edge test.  Both lists' places are known from the
// records, so one dependent read follows them: the longer list is staged in LDS (up to
// full_stage(HS, HP) words, from its overflow region or its head's inline entries) while the
// shorter one's entries are fetched into registers, then binary-searched.  The stage is 128
// words per request with heads of up to 32 words (8 KB per workgroup: 20 resident per CU, so
// config #2's ~2.8k dense waves run in one round; 256 words held 10 per CU and took two:
// 0.023 -> 0.017 ms per call) and 256 with 64-word heads, whose graphs' longer lists would
// otherwise be searched in global memory (config #3 shape: 7.1 vs 7.6e9 pipelined;
// profiles/r06/stage/)
__host__ __device__ constexpr uint32_t full_stage(int HS, int HP) { return HS >= 64 || HP >= 64 ? 256u : 128u; }
// Workgroup 0 also totals both lists' shard counts for the host (totals[0]: the rest list,
// totals[1]: this list), so the rest stage can be launched only when it has requests.
// Lean resident calls (plan label, timing events off, KETOGPU_LABEL_FUSE=1): the first
// stage and this pass run without statistics atomics (stats == nullptr: the statistics are
// diagnostics, collected by the same calls with events on), and workgroup 0 writes the two
// list totals straight into the host-mapped mirror (`mirror`: the words stats_reduce_kernel
// would write — zero statistics, spill counters {rest total, 0 ... 0, full total}), so the
// call needs no statistics launch and, after a call without rest requests, no clear.
template <int HS, int HP>
__global__ __launch_bounds__(64) void label_full_kernel(LabelGraph L, uint64_t *allowed, LabelRest R, LabelRest F,
                                                        unsigned int *total_rest, unsigned int *total_full,
                                                        unsigned long long *stats, unsigned long long *mirror) {
    constexpr uint32_t kFullStage = full_stage(HS, HP);
    __shared__ alignas(16) uint32_t stage[16][kFullStage];
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint32_t c = F.count[lane * kRestStride];
    const uint32_t nu = (c + 15) / 16;
    const uint32_t incl = wave_incl_sum_u32(nu);
    const uint64_t units = (uint64_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (blockIdx.x == 0) {
        const uint32_t tr = wave_sum_all(R.count[lane * kRestStride]), tf = wave_sum_all(c);
        if (lane == 0) *total_rest = tr, *total_full = tf;
        if (mirror && lane < 12)  // u32 spill counters at words 8..11: [0] rest total, [7] full total
            mirror[lane] = lane == 8 ? (unsigned long long)tr : lane == 11 ? (unsigned long long)tf << 32 : 0ull;
    }
    uint64_t ent = 0;
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint32_t shard = (uint32_t)__builtin_ctzll(__ballot(incl > u));
        const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)(incl - nu), (int)shard);
        const uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)shard);
        const uint64_t j = (u - first) * 16 + (lane & 15);
        uint4 r0 = make_uint4(KETOGPU_NODE_NONE, 0, 0, 0), r1 = make_uint4(0, 0, 0, 0);
        if (lane < 16 && j < cs) {
            const uint4 *rec = F.rec + 2 * (shard * F.cap + j);
            r0 = rec[0];
            r1 = rec[1];
        }
        const uint32_t idx = (uint32_t)__shfl((int)r0.x, (int)q, 64);
        const uint32_t rr = (uint32_t)__shfl((int)r0.y, (int)q, 64), tt = (uint32_t)__shfl((int)r0.z, (int)q, 64);
        const uint32_t ns = (uint32_t)__shfl((int)r0.w, (int)q, 64), np = (uint32_t)__shfl((int)r1.x, (int)q, 64);
        const uint32_t os = (uint32_t)__shfl((int)r1.y, (int)q, 64), op = (uint32_t)__shfl((int)r1.z, (int)q, 64);
        const bool valid = idx != KETOGPU_NODE_NONE;
        // each list: its overflow region when it overflows its head, else the head's entries
        const bool s_over = ns > (uint32_t)(HS - kHeadFixed), p_over = np > (uint32_t)(HP - kHeadFixed);
        const uint32_t *Sg = s_over ? L.S + (uint64_t)os * 16 : L.S + (uint64_t)tt * HS + kHeadFixed;
        const uint32_t *Pg = p_over ? L.P + (uint64_t)op * 16 : L.P + (uint64_t)rr * HP + kHeadFixed;
        const bool walk_p = np <= ns;
        const uint32_t nw = walk_p ? np : ns, nl = walk_p ? ns : np;
        const uint32_t *Lg = walk_p ? Sg : Pg, *W = walk_p ? Pg : Sg;
        // (16-byte units: an overflow region is 16-word aligned, a head's entries start 16
        // bytes into a 32-byte aligned head and are padded to a multiple of 4 words)
        {  // every staging load in flight before the LDS stores (a quad covers kFullStage words)
            constexpr int kSt = kFullStage / 16;  // 16-byte loads per lane
            const bool st = valid && nl <= kFullStage;
            uint4 v[kSt];
#pragma unroll
            for (int k = 0; k < kSt; k++) {
                const uint32_t i = sub + 4 * k;
                v[k] = st && i * 4 < nl ? reinterpret_cast<const uint4 *>(Lg)[i] : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int k = 0; k < kSt; k++) {
                const uint32_t i = sub + 4 * k;
                if (st && i * 4 < nl) reinterpret_cast<uint4 *>(stage[q])[i] = v[k];
            }
        }
        constexpr int kPre = 16;  // the walked entries this lane takes, fetched together
        uint32_t wk[kPre];
#pragma unroll
        for (int i = 0; i < kPre; i++) {
            const uint32_t k = sub + 4 * i;
            wk[i] = valid && k < nw ? W[k] : 0u;
        }
        wave_sync();
        const uint32_t *O = nl <= kFullStage ? stage[q] : Lg;
        bool hit = false;
        if (valid) {
#pragma unroll
            for (int i = 0; i < kPre; i++)
                if (!hit && sub + 4 * i < nw) hit = label_find_n(O, nl, wk[i]);
            for (uint32_t k = sub + 4 * kPre; k < nw && !hit; k += 4) hit = label_find_n(O, nl, W[k]);
            // the one-edge test: a non-interior root among S's raw entries (S the staged list
            // or the walked one; a landmark never equals a non-interior node id)
            if (sub == 0 && !hit && rr >= L.ni) hit = walk_p ? label_find_n(O, nl, rr) : label_find_n(W, nw, rr);
        }
        const uint64_t bits = __ballot(hit);
        if (valid && sub == 0) {
            if ((bits >> lane) & 0xF) atomicOr((unsigned long long *)&allowed[idx >> 6], 1ull << (idx & 63));
            ent += nl;  // the longer list read once more (u32 entries)
        }
        wave_sync();  // (the LDS rows are rewritten by the next unit)
    }
    const uint32_t e = wave_sum_all((uint32_t)ent);
    if (stats && lane == 0 && e) atomicAdd(&stat_slot(stats)[2], (unsigned long long)e);
}

// the second stage: plan lite's traversal over the requests the labels did not answer
// (in: request indices, *in_count of them, written by the first stage on this stream),
// gathered 16 to a unit; persistent over the listed requests.  A unit that outgrows its
// table lists its requests (out) for the multi-word global path (which also takes the
// wildcard roots).
template <class SH>
__global__ __launch_bounds__(64) void label_rest_kernel(DevGraph g, const FRec *frec, const FRec *brec,
                                                        const uint32_t *roots, const uint32_t *targets,
                                                        uint64_t *allowed, LabelRest R, unsigned int *total,
                                                        uint32_t *out, unsigned int *out_count,
                                                        unsigned long long *stats) {
    __shared__ SH S;
    // the shards' counts (lane k: shard k) and their units' exclusive prefix
    const uint32_t lane = threadIdx.x;
    const uint32_t c = R.count[lane * kRestStride];
    const uint32_t nu = (c + 15) / 16;
    const uint32_t incl = wave_incl_sum_u32(nu);
    const uint64_t units = (uint64_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t listed = wave_sum_all(c);  // (every lane: a wave-wide reduction)
    if (blockIdx.x == 0 && lane == 0) *total = listed;  // the host reads the total here (grid of the next call)
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        // the shard holding gathered unit u: the first whose inclusive prefix passes u
        const uint32_t shard = (uint32_t)__builtin_ctzll(__ballot(incl > u));
        const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)(incl - nu), (int)shard);
        const uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)shard);
        const uint64_t j = (u - first) * 16 + lane;
        uint32_t idx = KETOGPU_NODE_NONE, r = KETOGPU_NODE_NONE, t = KETOGPU_NODE_NONE;
        if (lane < 16 && j < cs) {
            idx = R.list[shard * R.cap + j];
            r = roots[idx];
            t = targets[idx];
        }
        lite_unit<SH, false>(S, g, frec, brec, bidi_load_rows(g, r, t), allowed, u, out, out_count, stats, nullptr,
                             idx, true);
        __syncthreads();
    }
}

// ----------------------------------------------------------------------- plan label: the heads' build
// The head arrays are built on the device from the 2-hop labels (built once per snapshot on
// the host, labels.cpp) and the graph already in HBM: one wave per node gathers the node's
// entries (S: Lin of the interior entries of rev(x) + its other entries; P: Lout(x) for an
// interior x, else Lout of every entry of fint(x)) into LDS, sorts them (bitonic over
// the 64 lanes) and drops duplicates.  A node with more than 64 entries before deduplication
// (or a row of more than 64) is left to the host (label_list), which writes its head after.
// Pass 1 counts (and a histogram picks the head size), a scan places the overflow lists,
// pass 2 writes.
struct LabelDevLists {
    const uint64_t *in_off, *out_off;
    const uint32_t *in, *out;
    const uint64_t *min, *mout;
    uint32_t Ni;
    uint32_t ph[3];  // a writable snapshot's placeholders (free slots: Df, Dbi, Dbo; else NONE)
};
constexpr uint32_t kLabelBig = 0xFFFFFFFEu;  // count of a node the host builds

// one node's list on the wave: v (one value per lane, ascending, duplicates and padding
// 0xFFFFFFFF not kept), keep (ballot of the kept lanes), mask; false: more than 64 entries
template <bool PSIDE>
__device__ __forceinline__ bool label_gather(const DevGraph &g, const LabelDevLists &D, uint32_t x, uint32_t *buf,
                                             uint32_t &v, uint64_t &keep, uint64_t &mask) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b = 0, m;
    bool synth = false;
    if constexpr (!PSIDE) {
        b = g.rev_off[x];
        m = g.rev_off[(uint64_t)x + 1] - b;
    } else if (x < D.Ni) {
        synth = true;  // the row is x itself: Lout(x)
        m = 1;
    } else {
        b = g.fint_off[x];
        m = g.fint_off[(uint64_t)x + 1] - b;
    }
    if (m > 64) return false;
    uint32_t e = KETOGPU_NODE_NONE, c = 0;
    uint64_t lo = 0, mk = 0;
    if (lane < m) {
        e = synth ? x : PSIDE ? g.fint_col[b + lane] : g.rev_col[b + lane];
        if (!synth && (e == D.ph[0] || e == D.ph[1] || e == D.ph[2])) {
            c = 0;  // a free slot (a row entry; an interior placeholder's own P head is Lout(x), as the host builds it)
        } else if (e < D.Ni) {
            const uint64_t *off = PSIDE ? D.out_off : D.in_off;
            lo = off[e];
            c = (uint32_t)(off[e + 1] - lo);
            mk = PSIDE ? D.mout[e] : D.min[e];
        } else {
            c = 1;
        }
    }
    const uint32_t incl = wave_incl_sum_u32(c);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (total > 64) return false;
    wave_sync();  // (the previous node's reads of buf are done)
    if (lane < m && c) {
        uint32_t o = incl - c;
        if (e < D.Ni) {
            const uint32_t *lst = (PSIDE ? D.out : D.in) + lo;
            for (uint32_t k = 0; k < c; k++) buf[o + k] = lst[k];
        } else {
            buf[o] = e;
        }
    }
    wave_sync();
    v = lane < total ? buf[lane] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 32; k; k >>= 1) mk |= __shfl_xor(mk, k, 64);
    mask = mk;
    // bitonic sort, ascending over the 64 lanes
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j; j >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v, (int)j, 64);
            const bool take_min = ((lane & j) == 0) == ((lane & k) == 0);
            v = take_min ? min(v, o) : max(v, o);
        }
    const uint32_t prev = (uint32_t)__shfl((int)v, (int)((lane + 63) & 63), 64);
    keep = __ballot(v != 0xFFFFFFFFu && (lane == 0 || v != prev));
    return true;
}

// pass 1: counts (kLabelBig for the host's nodes, listed in big), and per block the
// histogram hist = {non-empty, <= 4, <= 12, <= 28, <= 60 entries} (inline in heads of 8, 16,
// 32, 64 words)
template <bool PSIDE>
__global__ __launch_bounds__(256) void label_count_kernel(DevGraph g, LabelDevLists D, uint32_t n, uint32_t *cnt,
                                                          unsigned long long *hist, uint32_t *big,
                                                          unsigned int *big_n, uint32_t big_cap) {
    __shared__ uint32_t buf[4][64];
    __shared__ unsigned long long h[5];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < 5) h[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long hw[5] = {0, 0, 0, 0, 0};
    for (uint32_t x = blockIdx.x * 4 + wave; x < n; x += gridDim.x * 4) {
        uint32_t v;
        uint64_t keep, mask;
        if (!label_gather<PSIDE>(g, D, x, buf[wave], v, keep, mask)) {
            if (lane == 0) {
                cnt[x] = kLabelBig;
                const uint32_t at = atomicAdd(big_n, 1u);
                if (at < big_cap) big[at] = x;
            }
            continue;
        }
        const uint32_t c = (uint32_t)__popcll(keep);
        if (lane == 0) {
            cnt[x] = c;
            hw[0] += c != 0;
            hw[1] += c != 0 && c <= 4;
            hw[2] += c != 0 && c <= 12;
            hw[3] += c != 0 && c <= 28;
            hw[4] += c != 0 && c <= 60;
        }
    }
    if (lane == 0)
        for (int k = 0; k < 5; k++) atomicAdd(&h[k], hw[k]);
    __syncthreads();
    if (threadIdx.x < 5) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// overflow lists, in 16-word units: a list of more than cap entries takes ceil(count / 16)
__device__ __forceinline__ uint32_t label_ov16(uint32_t c, uint32_t cap) { return c > cap ? (c + 15) / 16 : 0u; }
constexpr uint32_t kLabelScanPer = 16, kLabelScanBlock = 256;  // nodes per thread, threads per block
// the scan's pass 1: each block's total of overflow units (its 4096 nodes)
__global__ __launch_bounds__(256) void label_ov_sum_kernel(const uint32_t *cnt, uint32_t n, uint32_t cap,
                                                           unsigned long long *block_sum) {
    __shared__ unsigned long long part[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * kLabelScanPer * kLabelScanBlock + threadIdx.x * kLabelScanPer;
    unsigned long long t = 0;
    for (uint32_t k = 0; k < kLabelScanPer; k++)
        if (b0 + k < n) t += label_ov16(cnt[b0 + k], cap);
#pragma unroll
    for (int k = 32; k; k >>= 1) t += __shfl_xor(t, k, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) block_sum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}
// pass 2: every node's overflow start (16-word units from base16) = the block's offset +
// the exclusive prefix within the block
__global__ __launch_bounds__(256) void label_ov_off_kernel(const uint32_t *cnt, uint32_t n, uint32_t cap,
                                                           const unsigned long long *block_off, uint64_t base16,
                                                           uint32_t *off16) {
    __shared__ unsigned long long part[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t b0 = (uint64_t)blockIdx.x * kLabelScanPer * kLabelScanBlock + threadIdx.x * kLabelScanPer;
    unsigned long long t = 0;
    for (uint32_t k = 0; k < kLabelScanPer; k++)
        if (b0 + k < n) t += label_ov16(cnt[b0 + k], cap);
    unsigned long long incl = t;  // inclusive scan over the wave
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const unsigned long long o = __shfl_up(incl, k, 64);
        if ((int)lane >= k) incl += o;
    }
    if (lane == 63) part[wave] = incl;
    __syncthreads();
    unsigned long long acc = base16 + block_off[blockIdx.x] + incl - t;
    for (uint32_t w = 0; w < wave; w++) acc += part[w];
    for (uint32_t k = 0; k < kLabelScanPer; k++)
        if (b0 + k < n) {
            const uint32_t c = cnt[b0 + k];
            off16[b0 + k] = label_ov16(c, cap) ? (uint32_t)acc : 0u;
            acc += label_ov16(c, cap);
        }
}

// pass 2: heads (and overflow lists) of every node the device counted; A is pre-filled
// with 0xFFFFFFFF
template <bool PSIDE>
__global__ __launch_bounds__(256) void label_write_kernel(DevGraph g, LabelDevLists D, uint32_t n, const uint32_t *cnt,
                                                          const uint32_t *off16, uint32_t *A, uint32_t H,
                                                          uint32_t permille, unsigned long long *tally) {
    __shared__ uint32_t buf[4][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long ent = 0, nol = 0, ovf = 0;  // (lane 0) entries, heads marked kNoLabel, overflow lists
    for (uint32_t x = blockIdx.x * 4 + wave; x < n; x += gridDim.x * 4) {
        uint32_t v;
        uint64_t keep, mask;
        if (!label_gather<PSIDE>(g, D, x, buf[wave], v, keep, mask)) continue;  // the host's node (wave-uniform)
        const uint32_t c = (uint32_t)__popcll(keep);
        uint32_t *head = A + (uint64_t)x * H;
        const bool inl = c <= H - kHeadFixed;
        if ((keep >> lane) & 1) {  // (an overflowing list: whole in the overflow region, its prefix in the head)
            const uint32_t pos = lanes_below(keep);
            if (pos < H - kHeadFixed) head[kHeadFixed + pos] = v;
            if (!inl) A[(uint64_t)off16[x] * 16 + pos] = v;
        }
        if (lane == 0) {
            // (the test knob's hash: labels.cpp label_nolabel)
            uint64_t hx = (uint64_t)x * 0x9E3779B97F4A7C15ull + 17;
            hx ^= hx >> 30, hx *= 0xbf58476d1ce4e5b9ull, hx ^= hx >> 27, hx *= 0x94d049bb133111ebull, hx ^= hx >> 31;
            const bool nolabel = !PSIDE && permille && c && hx % 1000 < permille;
            head[0] = nolabel ? kNoLabel : c;
            head[1] = inl ? 0u : off16[x];
            head[2] = (uint32_t)mask;
            head[3] = (uint32_t)(mask >> 32);
            ent += c;
            nol += nolabel;
            ovf += !inl;
        }
    }
    if (lane == 0) {
        atomicAdd(&tally[0], ent);
        atomicAdd(&tally[1], nol);
        atomicAdd(&tally[2], ovf);
    }
}

// big[i]'s overflow start and (in) count to the host; (out) counts of the host's nodes in
__global__ void label_big_io_kernel(const uint32_t *big, uint32_t nbig, uint32_t *cnt, const uint32_t *counts_in,
                                    const uint32_t *off16, uint32_t *off_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nbig) return;
    if (counts_in) cnt[big[i]] = counts_in[i];
    if (off16) off_out[i] = off16[big[i]];
}

// the host's nodes: packed records {node, count, H head words, the list when it overflows}
// (rec_off[i] = the i-th record's first word): heads to A + node * H, lists to the
// overflow start in the head's word 1
__global__ __launch_bounds__(64) void label_patch_kernel(const uint32_t *rec, const uint64_t *rec_off, uint32_t nrec,
                                                         uint32_t *A, uint32_t H) {
    for (uint32_t i = blockIdx.x; i < nrec; i += gridDim.x) {
        const uint32_t *r = rec + rec_off[i];
        const uint32_t x = r[0], c = r[1];
        uint32_t *head = A + (uint64_t)x * H;
        for (uint32_t k = threadIdx.x; k < H; k += 64) head[k] = r[2 + k];
        if (c > H - kHeadFixed) {
            uint32_t *dst = A + (uint64_t)r[3] * 16;
            for (uint32_t k = threadIdx.x; k < c; k += 64) dst[k] = r[2 + H + k];
        }
    }
}

// ----------------------------------------------------------------------- two-tier mode
// Kernels of the two-tier partitioned mode (tier.hpp, tier.cpp).  The evaluation is
// lite_unit over the rank's copy of the CORE (core_f / core_b: the rows among interior
// nodes, replicated) with seed rows that are either the rank's own rows read in place
// (world 1) or the rows the owners sent (recv, bounds per request): a seed's begins are
// offsets from core_f / core_b to the seed array (they may be "negative", i.e. wrap),
// which is all lite_unit needs to read them.
using TierStage1 = LiteShared<2048, 512, 512>;
using TierStage2 = LiteShared<8192, 1024, 1024>;

// owner and local index of global id v (shard.cpp layout: ids interleave the ranks inside
// each class range); NONE when another rank owns v or the slot is unused
__device__ __forceinline__ uint32_t tier_local(const tier::Graph &G, uint32_t v) {
    uint32_t base, l0, lim;
    if (v < G.Ni) {
        base = 0, l0 = 0, lim = G.Nil;
    } else if (v < G.Nx) {
        base = G.Ni, l0 = G.Nil, lim = G.Nxl;
    } else {
        base = G.Nx, l0 = G.Nxl, lim = G.Nl;
    }
    if (v >= G.N || (v - base) % G.world != G.rank) return KETOGPU_NODE_NONE;
    const uint32_t l = l0 + (v - base) / G.world;
    return l < lim ? l : KETOGPU_NODE_NONE;
}
__device__ __forceinline__ uint32_t tier_owner(const tier::Graph &G, uint32_t v) {
    const uint32_t base = v < G.Ni ? 0u : v < G.Nx ? G.Ni : G.Nx;
    return (v - base) % G.world;
}

// request c's ids, validated like validate_kernel (an id outside the layout: first_bad,
// and the request is answered false)
__device__ __forceinline__ void tier_request(const tier::Graph &G, const tier::Eval &E, uint64_t c, uint32_t &r,
                                             uint32_t &t) {
    r = t = KETOGPU_NODE_NONE;
    if (c >= E.n) return;
    r = E.roots[c];
    t = E.targets[c];
    if ((r != KETOGPU_NODE_NONE && r >= G.Nx) || (t != KETOGPU_NODE_NONE && t >= G.N)) {
        atomicMin(E.first_bad, (unsigned long long)c);
        r = t = KETOGPU_NODE_NONE;
    }
    if (t == KETOGPU_NODE_NONE) r = KETOGPU_NODE_NONE;
}

template <bool DIRECT>
__device__ __forceinline__ BidiSeed tier_seed(const tier::Graph &G, const tier::Eval &E, uint64_t unit) {
    BidiSeed s{KETOGPU_NODE_NONE, KETOGPU_NODE_NONE, 0, 0, 0, 0};
    if (threadIdx.x >= 16) return s;
    const uint64_t c = unit * 16 + threadIdx.x;
    tier_request(G, E, c, s.r, s.t);
    if (s.r == KETOGPU_NODE_NONE) return s;
    if constexpr (DIRECT) {
        const uint32_t lr = tier_local(G, s.r), lt = tier_local(G, s.t);
        uint64_t fb = 0, fe = 0, rb = 0, re = 0;
        if (lr != KETOGPU_NODE_NONE && lr < G.Nxl) fb = G.lf_off[lr], fe = G.lf_off[lr + 1];
        if (lt != KETOGPU_NODE_NONE) rb = G.lr_off[lt], re = G.lr_off[lt + 1];
        s.fb = (uint64_t)G.lf_base + fb;
        s.fe = (uint64_t)G.lf_base + fe;
        s.rb = (uint64_t)G.lr_base + rb;
        s.re = (uint64_t)G.lr_base + re;
    } else {
        const uint4 b = E.bnd[c];
        s.fb = (uint64_t)E.recv_base_f + b.x;
        s.fe = (uint64_t)E.recv_base_f + b.y;
        s.rb = (uint64_t)E.recv_base_b + b.z;
        s.re = (uint64_t)E.recv_base_b + b.w;
    }
    return s;
}

__device__ __forceinline__ DevGraph tier_devgraph(const tier::Graph &G) {
    DevGraph g{};
    g.Ni = G.Ni;
    g.Nx = G.Nx;
    g.N = G.N;
    g.both_max = G.both_max;
    g.seed_max = G.seed_max;
    g.seed_shift = 0;
    return g;
}

// stage 0: one unit per workgroup
template <class SH, bool DIRECT>
__global__ __launch_bounds__(64) void tier_eval_kernel(tier::Graph G, tier::Eval E, uint32_t *spill_out,
                                                       unsigned int *spill_count) {
    __shared__ SH S;
    const uint64_t unit = blockIdx.x;
    const DevGraph g = tier_devgraph(G);
    lite_unit<SH>(S, g, reinterpret_cast<const FRec *>(G.core_f), reinterpret_cast<const FRec *>(G.core_b),
                  tier_seed<DIRECT>(G, E, unit), E.allowed, unit, spill_out, spill_count, E.stats);
}

// stages 1 and 2: persistent over the previous stage's spilled units
template <class SH, bool DIRECT>
__global__ __launch_bounds__(64) void tier_cascade_kernel(tier::Graph G, tier::Eval E, const uint32_t *in_list,
                                                          const unsigned int *in_count, uint32_t *spill_out,
                                                          unsigned int *spill_count) {
    __shared__ SH S;
    const DevGraph g = tier_devgraph(G);
    const uint32_t cnt = *in_count;
    for (uint32_t b = blockIdx.x; b < cnt; b += gridDim.x) {
        const uint64_t unit = in_list[b];
        lite_unit<SH>(S, g, reinterpret_cast<const FRec *>(G.core_f), reinterpret_cast<const FRec *>(G.core_b),
                      tier_seed<DIRECT>(G, E, unit), E.allowed, unit, spill_out, spill_count, E.stats);
        __syncthreads();
    }
}

// queries of the batch: request i asks owner(r) for fint(r) (tag 2i) and owner(t) for
// rev(t) (tag 2i + 1).  Counting pass: per-destination totals (LDS histogram per block).
constexpr int kTB = 256;
__global__ __launch_bounds__(kTB) void tier_query_count_kernel(tier::Graph G, const uint32_t *roots,
                                                               const uint32_t *targets, uint64_t n,
                                                               unsigned long long *counts,
                                                               unsigned long long *first_bad, uint32_t *stage) {
    __shared__ unsigned int hist[64];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kTB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kTB) {
        const uint32_t r = roots[i], t = targets[i];
        if (stage) {  // one read of pinned host memory over PCIe; the later passes read HBM
            stage[i] = r;
            stage[n + i] = t;
        }
        if ((r != KETOGPU_NODE_NONE && r >= G.Nx) || (t != KETOGPU_NODE_NONE && t >= G.N)) {
            atomicMin(first_bad, (unsigned long long)i);
            continue;
        }
        if (r == KETOGPU_NODE_NONE || t == KETOGPU_NODE_NONE) continue;
        atomicAdd(&hist[tier_owner(G, r)], 1u);
        atomicAdd(&hist[tier_owner(G, t)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < G.world && hist[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
}

// scatter pass: per block, an LDS count per destination reserves one range per
// (block, destination) at the global cursor; lanes place their queries inside it
__global__ __launch_bounds__(kTB) void tier_query_scatter_kernel(tier::Graph G, const uint32_t *roots,
                                                                 const uint32_t *targets, uint64_t n,
                                                                 unsigned long long *cursor, tier::Query *out) {
    __shared__ unsigned int hist[64];
    __shared__ unsigned long long at[64];
    for (uint64_t i0 = (uint64_t)blockIdx.x * kTB; i0 < n; i0 += (uint64_t)gridDim.x * kTB) {
        if (threadIdx.x < 64) hist[threadIdx.x] = 0;
        __syncthreads();
        const uint64_t i = i0 + threadIdx.x;
        uint32_t r = KETOGPU_NODE_NONE, t = KETOGPU_NODE_NONE, dr = 0, dt = 0, pr = 0, pt = 0;
        bool ok = false;
        if (i < n) {
            r = roots[i];
            t = targets[i];
            ok = r != KETOGPU_NODE_NONE && t != KETOGPU_NODE_NONE && r < G.Nx && t < G.N;
        }
        if (ok) {
            dr = tier_owner(G, r);
            dt = tier_owner(G, t);
            pr = atomicAdd(&hist[dr], 1u);
            pt = atomicAdd(&hist[dt], 1u);
        }
        __syncthreads();
        if (threadIdx.x < G.world)
            at[threadIdx.x] = hist[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)hist[threadIdx.x]) : 0ull;
        __syncthreads();
        if (ok) {
            out[at[dr] + pr] = tier::Query{(uint32_t)(i << 1), r};
            out[at[dt] + pt] = tier::Query{(uint32_t)(i << 1 | 1), t};
        }
        __syncthreads();
    }
}

// world 1 (one owner): request i's queries sit at slots 2i and 2i + 1, no counting pass;
// a request without an answer (an id NONE or outside the layout) gets two NONE slots
__global__ __launch_bounds__(kTB) void tier_pair_kernel(tier::Graph G, const uint32_t *roots, const uint32_t *targets,
                                                        uint64_t n, tier::Query *out, unsigned long long *first_bad,
                                                        uint32_t *stage) {
    for (uint64_t i = (uint64_t)blockIdx.x * kTB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kTB) {
        uint32_t r = roots[i], t = targets[i];
        if (stage) {
            stage[i] = r;
            stage[n + i] = t;
        }
        if ((r != KETOGPU_NODE_NONE && r >= G.Nx) || (t != KETOGPU_NODE_NONE && t >= G.N)) {
            atomicMin(first_bad, (unsigned long long)i);
            r = t = KETOGPU_NODE_NONE;
        }
        if (r == KETOGPU_NODE_NONE || t == KETOGPU_NODE_NONE) r = t = KETOGPU_NODE_NONE;
        reinterpret_cast<uint4 *>(out)[i] = make_uint4((uint32_t)(i << 1), r, (uint32_t)(i << 1 | 1), t);
    }
}

// the owner's side: the length of the row each received query asks for (lens[j]); a
// query for a node this rank does not own (a misrouted record) raises *bad
__device__ __forceinline__ void tier_row(const tier::Graph &G, const tier::Query &q, uint64_t &b, uint64_t &e,
                                         bool &bad) {
    b = e = 0;
    bad = false;
    if (q.node == KETOGPU_NODE_NONE) return;  // a world-1 pair slot of an unanswerable request
    const uint32_t l = tier_local(G, q.node);
    if (l == KETOGPU_NODE_NONE) {
        bad = true;
        return;
    }
    if (G.label) {  // label mode: the node's S / P list (masks, then entries)
        const uint64_t *o = (q.tag & 1u) ? G.ls_off : l < G.Nxl ? G.lp_off : nullptr;
        if (o) b = o[l], e = o[l + 1];
        return;
    }
    if (q.tag & 1u) {
        b = G.lr_off[l];
        e = G.lr_off[l + 1];
    } else if (l < G.Nxl) {
        b = G.lf_off[l];
        e = G.lf_off[l + 1];
    }
}

// srcb (may be null): each row's / list's first entry too, so the copy pass reads it
// sequentially instead of looking the owned node's offsets up again
__global__ __launch_bounds__(kTB) void tier_reply_len_kernel(tier::Graph G, const tier::Query *q, uint64_t n,
                                                             uint64_t *lens, unsigned long long *bad, uint64_t *srcb) {
    for (uint64_t j = (uint64_t)blockIdx.x * kTB + threadIdx.x; j < n; j += (uint64_t)gridDim.x * kTB) {
        uint64_t b, e;
        bool miss;
        tier_row(G, q[j], b, e, miss);
        if (miss) atomicMin(bad, (unsigned long long)j);
        lens[j] = e - b;
        if (srcb) srcb[j] = b;
    }
}

// exclusive scan of u64 in place over tiles of kTB * 4: tile sums, the sums' scan (one
// block), then each tile scanned with its offset; v[n] = the total
constexpr int kScanTile = kTB * 4;
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t x, uint64_t *tmp, uint64_t &total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan(x, lane);
    if (lane == 63) tmp[wv] = incl;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
    for (int w = 0; w < kTB / 64; w++) {
        if (w < wv) before += tmp[w];
        total += tmp[w];
    }
    __syncthreads();
    return before + incl - x;
}
__global__ __launch_bounds__(kTB) void tier_scan_sums_kernel(const uint64_t *v, uint64_t n, uint64_t *sums) {
    __shared__ uint64_t tmp[kTB / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * 4;
    uint64_t x = 0;
    for (int k = 0; k < 4; k++)
        if (base + k < n) x += v[base + k];
    uint64_t total;
    block_excl_scan(x, tmp, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}
__global__ __launch_bounds__(kTB) void tier_scan_top_kernel(uint64_t *sums, uint64_t nb) {
    __shared__ uint64_t tmp[kTB / 64];
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += kTB) {
        const uint64_t i = b0 + threadIdx.x;
        const uint64_t x = i < nb ? sums[i] : 0;
        uint64_t total;
        const uint64_t ex = block_excl_scan(x, tmp, total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) sums[nb] = carry;
}
__global__ __launch_bounds__(kTB) void tier_scan_tiles_kernel(uint64_t *v, uint64_t n, const uint64_t *sums, uint64_t nb) {
    __shared__ uint64_t tmp[kTB / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * 4;
    uint64_t x[4], s = 0;
    for (int k = 0; k < 4; k++) {
        x[k] = base + k < n ? v[base + k] : 0;
        s += x[k];
    }
    uint64_t total;
    uint64_t run = sums[blockIdx.x] + block_excl_scan(s, tmp, total);
    for (int k = 0; k < 4; k++) {
        if (base + k < n) v[base + k] = run;
        run += x[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) v[n] = sums[nb];
}

// the replies: one wave per 64 queries writes their rows as consecutive records (each
// output index finds its query by a binary search over the wave's offsets in LDS, so
// consecutive lanes write consecutive records), pad = the query's tag
__global__ __launch_bounds__(kTB) void tier_reply_copy_kernel(tier::Graph G, const tier::Query *q, uint64_t n,
                                                              const uint64_t *off, tier::Reply *out, uint64_t cap) {
    __shared__ uint64_t s_pre[kTB / 64][65];
    __shared__ uint64_t s_src[kTB / 64][64];
    __shared__ uint32_t s_tag[kTB / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t j0 = ((uint64_t)blockIdx.x * (kTB / 64) + wv) * 64; j0 < n; j0 += (uint64_t)gridDim.x * kTB) {
        const uint64_t j = j0 + lane;
        uint64_t b = 0, e = 0;
        uint32_t tag = 0;
        if (j < n) {
            bool miss;
            tier_row(G, q[j], b, e, miss);
            tag = q[j].tag;
        }
        const uint64_t o0 = off[j0];
        s_pre[wv][lane] = (j < n ? off[j] : off[n]) - o0;
        s_src[wv][lane] = b;
        s_tag[wv][lane] = tag;
        const uint64_t total = (j0 + 64 < n ? off[j0 + 64] : off[n]) - o0;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        for (uint64_t o = lane; o < total; o += 64) {
            int lo = 0, hi = 64;  // the last query whose offset is <= o owns it (empty rows never win)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_pre[wv][mid] <= o)
                    lo = mid;
                else
                    hi = mid;
            }
            const uint32_t tg = s_tag[wv][lo];
            const uint32_t *src = (tg & 1u) ? G.lr_node : G.lf_node;  // 4 bytes per entry, not the 16-byte record
            const uint32_t node = src[s_src[wv][lo] + (o - s_pre[wv][lo])];
            if (o0 + o < cap) out[o0 + o] = tier::Reply{node, tg};
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// received replies -> seed records (entry x: its core row in this rank's copy of the core —
// forward entries are interior; a backward entry outside the interior is (x, 0, 0): only
// compared with the root) and per request seed bounds (each query's row is contiguous).
// Lane-consecutive entries: a wave's 64 lanes read 64 consecutive 8-byte replies and write
// 64 consecutive 16-byte records per instruction (1 KB, whole lines; with four consecutive
// entries per lane each store instruction wrote 16 of every 64 bytes: PMC 406 MB written
// per 10^6 config-#5 requests for 298 MB of records).  The neighbours' tags that decide
// the bounds come from the adjacent lanes (the wave's first / last lane reads them).  The
// random reads into the core's row table are L2 requests, one per lane.
constexpr int kSeedPer = 4;
__global__ __launch_bounds__(kTB) void tier_seed_kernel(tier::Graph G, const tier::Reply *recv, uint64_t n,
                                                        tier::Rec *seed, uint4 *bnd, uint64_t nreq) {
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint64_t span = (uint64_t)kTB * kSeedPer;  // entries per workgroup pass
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        tier::Reply e[kSeedPer];
        uint2 row[kSeedPer];
#pragma unroll
        for (int j = 0; j < kSeedPer; j++) {
            const uint64_t k = base + (uint64_t)j * kTB + threadIdx.x;
            e[j] = k < n ? recv[k] : tier::Reply{~0u, ~0u};
        }
#pragma unroll
        for (int j = 0; j < kSeedPer; j++) {
            const uint64_t k = base + (uint64_t)j * kTB + threadIdx.x;
            const uint2 *rows = (e[j].tag & 1u) ? G.core_b_row : G.core_f_row;
            const bool in = k < n && e[j].node < G.Ni;
            row[j] = in ? rows[e[j].node] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < kSeedPer; j++) {
            const uint64_t k = base + (uint64_t)j * kTB + threadIdx.x;
            const uint32_t tag = e[j].tag;
            uint32_t prev = (uint32_t)__shfl_up((int)tag, 1, 64), next = (uint32_t)__shfl_down((int)tag, 1, 64);
            if (lane == 0) prev = k && k - 1 < n ? recv[k - 1].tag : ~0u;
            if (lane == 63) next = k + 1 < n ? recv[k + 1].tag : ~0u;
            if (k >= n) continue;
            if (k + 1 >= n) next = ~0u;
            seed[k] = tier::Rec{e[j].node, row[j].y, row[j].x, tag};
            const uint64_t i = tag >> 1;
            if (i >= nreq) continue;
            uint32_t *b = reinterpret_cast<uint32_t *>(&bnd[i]) + 2 * (tag & 1u);
            if (prev != tag) b[0] = (uint32_t)k;
            if (next != tag) b[1] = (uint32_t)(k + 1);
        }
    }
}

// Label mode replies (tier.hpp "label replies"): a destination's segment is the lengths of
// the lists it asked for, in its query order, then the lists themselves, 4-byte words.
// seg(k): the segment of query k, given the segments' first queries (world + 1 entries)
__device__ __forceinline__ uint32_t tier_seg(const uint64_t *first, uint32_t world, uint64_t k) {
    uint32_t lo = 0, hi = world;  // the last p with first[p] <= k
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] <= k)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// The owner's side: query j of segment p (qs: the received segments' first queries, off:
// the lists' lengths scanned over all received queries) writes its length at
// j + off[qs[p]] and its list at qs[p + 1] + off[j] — the segment layout above, with no
// per-segment pass.  One wave per 64 queries, lanes over consecutive words (like
// tier_reply_copy_kernel), eight words per lane in flight.  bnd (world 1, may be null): the
// asker is this rank and its layout this one, so each query also writes its request's list
// bounds (tier_label_bounds_kernel's result, no separate pass and no clearing: every request
// has both slots)
__global__ __launch_bounds__(kTB) void tier_label_reply_kernel(tier::Graph G, const tier::Query *q, uint64_t n,
                                                               const uint64_t *off, const uint64_t *srcb, const uint64_t *qs,
                                                               uint32_t world, uint32_t *out, uint64_t cap, uint4 *bnd,
                                                               uint64_t nreq) {
    __shared__ uint64_t s_pre[kTB / 64][65];
    __shared__ uint64_t s_src[kTB / 64][64];
    __shared__ uint64_t s_dst[kTB / 64][64];
    __shared__ uint32_t s_side[kTB / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t j0 = ((uint64_t)blockIdx.x * (kTB / 64) + wv) * 64; j0 < n; j0 += (uint64_t)gridDim.x * kTB) {
        const uint64_t j = j0 + lane;
        uint64_t b = 0, e = 0, dst = 0;
        uint32_t side = 0;
        if (j < n) {
            const tier::Query qq = q[j];
            b = srcb[j];  // (tier_reply_len_kernel's lookup of the list)
            e = b + (off[j + 1] - off[j]);
            side = qq.tag & 1u;
            // (world 1: one segment, qs = {0, n} — not read from memory)
            const uint32_t p = world == 1 ? 0u : tier_seg(qs, world, j);
            const uint64_t q0 = world == 1 ? 0 : qs[p], q1 = world == 1 ? n : qs[p + 1];
            const uint64_t h = j + off[q0];
            if (h < cap) out[h] = (uint32_t)(e - b);
            dst = q1 + off[j];
            if (bnd && (qq.tag >> 1) < nreq) {
                const uint64_t end = dst + (e - b);
                reinterpret_cast<uint2 *>(&bnd[qq.tag >> 1])[side] =
                    end <= cap ? make_uint2((uint32_t)dst, (uint32_t)end) : make_uint2(0u, 0u);
            }
        }
        const uint64_t o0 = off[j0];
        s_pre[wv][lane] = (j < n ? off[j] : off[n]) - o0;
        s_src[wv][lane] = b;
        s_dst[wv][lane] = dst;
        s_side[wv][lane] = side;
        const uint64_t total = (j0 + 64 < n ? off[j0 + 64] : off[n]) - o0;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        constexpr int kU = 8;  // words per lane in flight
        for (uint64_t ob = 0; ob < total; ob += 64 * kU) {
            uint32_t v[kU];
            uint64_t d[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const uint64_t o = ob + 64 * u + lane;
                d[u] = ~0ull;
                v[u] = 0;
                if (o < total) {
                    int lo = 0, hi = 64;  // the last query whose offset is <= o owns it (empty lists never win)
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (s_pre[wv][mid] <= o)
                            lo = mid;
                        else
                            hi = mid;
                    }
                    const uint64_t w = o - s_pre[wv][lo];
                    const uint32_t *src = s_side[wv][lo] ? G.ls_col : G.lp_col;
                    d[u] = s_dst[wv][lo] + w;
                    v[u] = src[s_src[wv][lo] + w];
                }
            }
#pragma unroll
            for (int u = 0; u < kU; u++)
                if (d[u] < cap) out[d[u]] = v[u];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// The asker's side: the length of the list its k-th sent query got back (sq: its sent
// segments' first queries, rp: the received segments' first words)
__global__ __launch_bounds__(kTB) void tier_label_lens_kernel(const uint32_t *recv, uint64_t nsent, const uint64_t *sq,
                                                              const uint64_t *rp, uint32_t world, uint64_t *lens) {
    for (uint64_t k = (uint64_t)blockIdx.x * kTB + threadIdx.x; k < nsent; k += (uint64_t)gridDim.x * kTB) {
        const uint32_t p = tier_seg(sq, world, k);
        lens[k] = recv[rp[p] + (k - sq[p])];
    }
}

// ... and with the lengths scanned (g), each list's bounds: it starts at sq[p + 1] + g[k]
// (the same layout seen from the asker), for request tag >> 1, side tag & 1.  A list that
// would end past the received words (cap) is left empty, so the evaluation never reads
// past them (the world-1 step evaluates a batch whose replies outgrew the buffer again)
__global__ __launch_bounds__(kTB) void tier_label_bounds_kernel(const tier::Query *sent, uint64_t nsent,
                                                                const uint64_t *sq, const uint64_t *g, uint32_t world,
                                                                uint4 *bnd, uint64_t nreq, uint64_t cap) {
    for (uint64_t k = (uint64_t)blockIdx.x * kTB + threadIdx.x; k < nsent; k += (uint64_t)gridDim.x * kTB) {
        const uint32_t p = tier_seg(sq, world, k);
        const uint32_t tag = sent[k].tag;
        const uint64_t i = tag >> 1;
        if (i >= nreq) continue;
        const uint64_t b = sq[p + 1] + g[k], e = b + (g[k + 1] - g[k]);
        reinterpret_cast<uint2 *>(&bnd[i])[tag & 1u] = e <= cap ? make_uint2((uint32_t)b, (uint32_t)e) : make_uint2(0u, 0u);
    }
}

// Label mode evaluation: one wave per 16 requests, four lanes per request.  Both lists'
// first kTierLab words go to LDS; the masks decide first, then the shorter list's entries
// (round-robin over the four lanes) are binary-searched in the longer one (LDS when it fits,
// else where it lies).  DIRECT: world 1, the lists read in place.
constexpr uint32_t kTierLab = 64;
template <bool DIRECT>
__global__ __launch_bounds__(64) void tier_label_kernel(tier::Graph G, tier::Eval E, const uint32_t *recv) {
    __shared__ uint32_t L[16][2][kTierLab];
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint64_t c = (uint64_t)blockIdx.x * 16 + q;
    uint32_t r = KETOGPU_NODE_NONE, t = KETOGPU_NODE_NONE;
    // exchange mode: the query passes validated the ids (first_bad) and sent nothing for a
    // request without an answer (its bounds stay empty): the bounds are the first read
    if constexpr (DIRECT) tier_request(G, E, c, r, t);
    const uint32_t *lp = nullptr, *ls = nullptr;
    uint32_t np = 0, ns = 0;
    if (DIRECT ? r != KETOGPU_NODE_NONE : c < E.n) {
        if constexpr (DIRECT) {
            const uint32_t lr = tier_local(G, r), lt = tier_local(G, t);
            if (lr != KETOGPU_NODE_NONE && lr < G.Nxl) {
                const uint64_t b = G.lp_off[lr];
                lp = G.lp_col + b;
                np = (uint32_t)(G.lp_off[lr + 1] - b);
            }
            if (lt != KETOGPU_NODE_NONE) {
                const uint64_t b = G.ls_off[lt];
                ls = G.ls_col + b;
                ns = (uint32_t)(G.ls_off[lt + 1] - b);
            }
        } else {
            const uint4 b = E.bnd[c];
            lp = recv + b.x;
            np = b.y - b.x;
            ls = recv + b.z;
            ns = b.w - b.z;
        }
    }
    {  // both lists' first kTierLab words, every load in flight before the LDS stores
        constexpr int kStg = kTierLab / 4;
        uint32_t vp[kStg], vs[kStg];
#pragma unroll
        for (int i = 0; i < kStg; i++) {
            const uint32_t j = sub + 4 * i;
            vp[i] = j < np ? lp[j] : 0u;
            vs[i] = j < ns ? ls[j] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kStg; i++) {
            const uint32_t j = sub + 4 * i;
            if (j < np) L[q][0][j] = vp[i];
            if (j < ns) L[q][1][j] = vs[i];
        }
    }
    __syncthreads();
    bool hit = false;
    const bool valid = np >= 2 && ns >= 2;
    if (valid) {
        const uint64_t pm = L[q][0][0] | (uint64_t)L[q][0][1] << 32, sm = L[q][1][0] | (uint64_t)L[q][1][1] << 32;
        hit = (pm & sm) != 0;
        // walk A (the shorter), search B
        const bool a_p = np <= ns;
        const uint32_t na = (a_p ? np : ns) - 2, nb = (a_p ? ns : np) - 2;
        const uint32_t *A = a_p ? &L[q][0][0] : &L[q][1][0], *B = a_p ? &L[q][1][0] : &L[q][0][0];
        const uint32_t *Ag = a_p ? lp : ls, *Bg = a_p ? ls : lp;
        for (uint32_t k = sub; k < na && !hit; k += 4) {
            const uint32_t x = k + 2 < kTierLab ? A[k + 2] : Ag[k + 2];
            hit = label_find_n(nb + 2 <= kTierLab ? B + 2 : Bg + 2, nb, x);
        }
    }
    const uint64_t hb = __ballot(hit);
    uint64_t bits = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) bits |= ((hb >> (4 * k)) & 0xFull) ? (1ull << k) : 0ull;
    const uint64_t vb = __ballot(valid && sub == 0);
    uint32_t ent = sub == 0 ? np + ns : 0;
    for (int o = 32; o; o >>= 1) ent += (uint32_t)__shfl_xor((int)ent, o, 64);
    if (lane == 0) {
        // the unit's 16 answers are the 16-bit word blockIdx.x of the answer array: a plain
        // store (zeros included, the last word's tail zeroed), so the array needs no clearing
        reinterpret_cast<uint16_t *>(E.allowed)[blockIdx.x] = (uint16_t)bits;
        if (blockIdx.x + 1 == gridDim.x)
            for (uint32_t u = gridDim.x; u < (gridDim.x + 3) / 4 * 4; u++) reinterpret_cast<uint16_t *>(E.allowed)[u] = 0;
        if (vb) {
            atomicAdd(&stat_slot(E.stats)[0], 2ull * (unsigned long long)__popcll(vb));
            atomicAdd(&stat_slot(E.stats)[1], (unsigned long long)ent);
        }
    }
}

// bad (may be null): a host batch's first-invalid-request word, reset to "none" here
// instead of by a separate memset launch
__global__ __launch_bounds__(kBlock) void clear_kernel(uint64_t *a, uint64_t na, uint64_t *b, uint64_t nb,
                                                       unsigned long long *c, uint64_t nc, unsigned long long *bad) {
    if (bad && blockIdx.x == 0 && threadIdx.x == 0) *bad = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < na + nb + nc; i += (uint64_t)gridDim.x * kBlock) {
        if (i < na)
            a[i] = 0;
        else if (i < na + nb)
            b[i - na] = 0;
        else
            c[i - na - nb] = 0;
    }
}

// Device-side request validation (no host pass over the batch): an id outside the
// snapshot becomes NONE before any traversal kernel reads it, and the smallest such
// request index is recorded; the call then fails with KETOGPU_EINVAL.
__global__ __launch_bounds__(kBlock) void validate_kernel(uint32_t *roots, uint32_t *targets, uint64_t n, uint32_t Nx,
                                                          uint32_t N, uint64_t base, unsigned long long *first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = roots[i], t = targets[i];
    if ((r != KETOGPU_NODE_NONE && r >= Nx) || (t != KETOGPU_NODE_NONE && t >= N)) {
        roots[i] = KETOGPU_NODE_NONE;
        targets[i] = KETOGPU_NODE_NONE;
        atomicMin(first_bad, (unsigned long long)(base + i));
    }
}

// The chunk's requests read straight from pinned host memory (device-accessible, zero
// copy over PCIe), validated as validate_kernel does and stored in HBM: no DMA copy per
// chunk (each costs ~20 us of setup on the copy engine, two per chunk) and no separate
// validation launch.
__global__ __launch_bounds__(kBlock) void load_kernel(const uint32_t *hr, const uint32_t *ht, uint64_t c0, uint64_t m,
                                                      uint32_t *dr, uint32_t *dt, uint32_t Nx, uint32_t N,
                                                      unsigned long long *first_bad) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < m; i += (uint64_t)gridDim.x * kBlock) {
        uint32_t r = hr[c0 + i], t = ht[c0 + i];
        if ((r != KETOGPU_NODE_NONE && r >= Nx) || (t != KETOGPU_NODE_NONE && t >= N)) {
            atomicMin(first_bad, (unsigned long long)(c0 + i));
            r = t = KETOGPU_NODE_NONE;
        }
        dr[c0 + i] = r;
        dt[c0 + i] = t;
    }
}

// The run's results in one launch into pinned host memory: result words, flag words (when
// wanted) and the first invalid request index — instead of one DMA copy each.
// out_bits (may be null): the result words go to the caller's own pinned buffer instead
__global__ __launch_bounds__(kBlock) void emit_kernel(const uint64_t *allowed, const uint64_t *flags, uint64_t words,
                                                      const unsigned long long *first_bad, uint64_t *out,
                                                      uint64_t *out_bits) {
    const uint64_t nf = flags ? words : 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < words + nf + 1; i += (uint64_t)gridDim.x * kBlock) {
        if (i < words && out_bits)
            out_bits[i] = allowed[i];
        else
            out[i] = i < words ? allowed[i] : i < words + nf ? flags[i - words] : (uint64_t)*first_bad;
    }
}

// sum the spread statistics slots of `regions` regions into out[3 * region + k]
// mirror (host-mapped pinned memory, may be null): out[0, mirror_words) is also written
// there, so the host reads the statistics and the spill counters after its one
// synchronization without a separate copy
// Blocks >= 1 (when E.out is set): the host batch's emit (emit_kernel's work) in the same
// launch, one launch less at the end of every host-to-host call.
struct EmitReq {
    const uint64_t *allowed = nullptr, *flags = nullptr;
    uint64_t words = 0;
    const unsigned long long *first_bad = nullptr;
    uint64_t *out = nullptr;
    uint64_t *out_bits = nullptr;  // the caller's own pinned result words (else out[0, words))
};
__global__ __launch_bounds__(kBlock) void stats_reduce_kernel(const unsigned long long *slots, int regions,
                                                              unsigned long long *out, unsigned long long *mirror,
                                                              int mirror_words, EmitReq E) {
    if (blockIdx.x) {
        const uint64_t nf = E.flags ? E.words : 0, m = E.words + nf + 1;
        for (uint64_t i = (uint64_t)(blockIdx.x - 1) * kBlock + threadIdx.x; i < m; i += (uint64_t)(gridDim.x - 1) * kBlock)
            if (i < E.words && E.out_bits)
                E.out_bits[i] = E.allowed[i];
            else
                E.out[i] = i < E.words ? E.allowed[i] : i < E.words + nf ? E.flags[i - E.words] : (uint64_t)*E.first_bad;
        return;
    }
    __shared__ unsigned long long part[kBlock / 64][3];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int r = 0; r < regions; r++) {
        unsigned long long v[3] = {0, 0, 0};
        for (int i = threadIdx.x; i < kStatSlots; i += kBlock)
            for (int k = 0; k < 3; k++) v[k] += slots[(size_t)r * 4 * kStatSlots + (size_t)i * 4 + k];
        for (int k = 0; k < 3; k++) {
            for (int d = 32; d; d >>= 1) v[k] += __shfl_down(v[k], d, 64);
            if (lane == 0) part[wv][k] = v[k];
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            unsigned long long t = 0;
            for (int w = 0; w < kBlock / 64; w++) t += part[w][threadIdx.x];
            out[3 * r + threadIdx.x] = t;
        }
        __syncthreads();
    }
    __threadfence_block();
    if (mirror && (int)threadIdx.x < mirror_words) mirror[threadIdx.x] = out[threadIdx.x];
}

// ------------------------------------------------- wave-synchronous units
// Same algorithm as unit_kernel with ONE WAVE per unit: the four waves of a workgroup
// own four independent LDS partitions, so a BFS level needs no workgroup barrier, only
// in-order wave execution (wave_sync orders the LDS traffic between phases).

template <int U, int HLOG>
struct WaveLDS {
    static constexpr int H = 1 << HLOG;
    static constexpr int F = H / 2;  // frontier list capacity
    uint32_t key[H];
    uint32_t st[H];  // visited bits [0, U) | pending bits [16, 16 + U)
    uint16_t cur_slot[F], nxt_slot[F], cur_mask[F];
    uint64_t c_begin[64];
    uint32_t c_pre[65];
    uint16_t c_mask[64];
    uint32_t root[U], target[U];
    uint32_t n_used, n_nxt, spill, pad;
};

template <int U, int HLOG>
__device__ __forceinline__ uint32_t wslot(uint32_t u) {
    return (u * 2654435761u) >> (32 - HLOG);
}

template <int U, int HLOG>
__device__ __forceinline__ void wave_push(const DevGraph &g, WaveLDS<U, HLOG> &S, bool want, uint32_t u, uint32_t m,
                                          const uint32_t *has_kids, uint64_t *flag_word, int shift, int lane) {
    constexpr int H = 1 << HLOG;
    int h = -1;
    bool inserted = false;
    if (want) {
        uint32_t hh = wslot<U, HLOG>(u);
        for (int p = 0; p < H; p++, hh = (hh + 1) & (H - 1)) {
            uint32_t kv = S.key[hh];
            if (kv == kEmpty) {
                uint32_t prev = atomicCAS(&S.key[hh], kEmpty, u);
                if (prev == kEmpty) {
                    inserted = true;
                    h = (int)hh;
                    break;
                }
                kv = prev;
            }
            if (kv == u) {
                h = (int)hh;
                break;
            }
        }
        if (h < 0) S.spill = 1;
    }
    uint64_t bal = __ballot(inserted);
    if (bal && lane == 0) {
        uint32_t c = (uint32_t)__popcll(bal);
        if (atomicAdd(&S.n_used, c) + c > (uint32_t)(H * 3 / 4)) S.spill = 1;
    }
    bool app = false;
    if (h >= 0) {
        uint32_t old = atomicOr(&S.st[h], m);
        uint32_t newly = m & ~old & ((1u << U) - 1);
        if (newly) {
            if (g.row_amb && bit_of(g.row_amb, u))
                atomicOr((unsigned long long *)flag_word, (unsigned long long)newly << shift);
            if (bit_of(has_kids, u)) {
                uint32_t o2 = atomicOr(&S.st[h], newly << 16);
                app = !(o2 >> 16);
            }
        }
    }
    uint64_t ab = __ballot(app);
    if (ab) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&S.n_nxt, (uint32_t)__popcll(ab));
        base = __shfl(base, 0, 64);
        uint32_t idx = base + (uint32_t)__popcll(ab & ((1ull << lane) - 1));
        if (app) {
            if (idx < (uint32_t)WaveLDS<U, HLOG>::F)
                S.nxt_slot[idx] = (uint16_t)h;
            else
                S.spill = 1;
        }
    }
}

// expand up to 64 entries held by the lanes (lane < k: node v, mask m); all lanes call
template <int U, int HLOG>
__device__ __forceinline__ void wave_expand(const DevGraph &g, WaveLDS<U, HLOG> &S, uint32_t k, bool have, uint32_t v,
                                            uint32_t m, const uint32_t *has_kids, uint64_t *flag_word, int shift,
                                            int lane, uint64_t &rows, uint64_t &edges) {
    uint32_t d = 0;
    uint64_t b = 0;
    if (have) {
        b = g.fint_off[v];
        d = (uint32_t)(g.fint_off[v + 1] - b);
        rows++;
    }
    uint32_t x = d;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        uint32_t t = __shfl_up(x, s, 64);
        if (lane >= s) x += t;
    }
    uint32_t total = __shfl(x, 63, 64);
    S.c_begin[lane] = b;
    S.c_pre[lane] = x - d;
    S.c_mask[lane] = (uint16_t)m;
    wave_sync();
    for (uint32_t base = 0; base < total; base += 64) {
        uint32_t e = base + lane;
        bool want = e < total;
        uint32_t u = 0, mm = 0;
        if (want) {
            uint32_t lo = 0, hi = k;
            while (hi - lo > 1) {
                uint32_t mid = (lo + hi) >> 1;
                if (S.c_pre[mid] <= e)
                    lo = mid;
                else
                    hi = mid;
            }
            u = g.fint_col[S.c_begin[lo] + (e - S.c_pre[lo])];
            mm = S.c_mask[lo];
            edges++;
        }
        wave_push<U, HLOG>(g, S, want, u, mm, has_kids, flag_word, shift, lane);
    }
    wave_sync();
}

template <int U, int HLOG>
__global__ __launch_bounds__(kBlock) void wave_unit_kernel(DevGraph g, const uint32_t *has_kids, const uint32_t *roots,
                                                           const uint32_t *targets, uint64_t n, uint64_t *allowed,
                                                           uint64_t *flags, uint32_t *spill_out,
                                                           unsigned int *spill_count, unsigned long long *stats) {
    using L = WaveLDS<U, HLOG>;
    constexpr int H = L::H;
    __shared__ L lds[kBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    L &S = lds[wv];
    const uint64_t unit = (uint64_t)blockIdx.x * (kBlock / 64) + wv;
    const uint64_t c0 = unit * U;
    if (c0 >= n) return;
    uint64_t *flag_word = &flags[c0 >> 6];
    const int shift = (int)(c0 & 63);
    const unsigned long long unit_bits = ((1ull << U) - 1) << shift;
    for (int i = lane; i < H; i += 64) {
        S.key[i] = kEmpty;
        S.st[i] = 0;
    }
    if (lane == 0) S.n_used = S.n_nxt = S.spill = 0;
    bool dyn = false;
    uint32_t r = KETOGPU_NODE_NONE;
    if (lane < U) {
        uint64_t c = c0 + lane;
        uint32_t t = KETOGPU_NODE_NONE;
        if (c < n) {
            r = roots[c];
            t = targets[c];
        }
        if (t == KETOGPU_NODE_NONE) r = KETOGPU_NODE_NONE;
        dyn = r != KETOGPU_NODE_NONE && r >= kDynBase;
        S.root[lane] = r;
        S.target[lane] = t;
    }
    if (__ballot(dyn)) {
        if (lane == 0) spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
        return;
    }
    wave_sync();
    uint64_t rows = 0, edges = 0, rev = 0;
    {
        bool have = lane < U && r != KETOGPU_NODE_NONE;
        if (have && g.row_amb && bit_of(g.row_amb, r))
            atomicOr((unsigned long long *)flag_word, (unsigned long long)1 << (shift + lane));
        wave_expand<U, HLOG>(g, S, U, have, r, 1u << (lane & 31), has_kids, flag_word, shift, lane, rows, edges);
    }
    for (;;) {
        uint32_t cnt = S.n_nxt;
        if (S.spill || !cnt) break;
        for (uint32_t i = lane; i < cnt; i += 64) {
            uint16_t s = S.nxt_slot[i];
            S.cur_slot[i] = s;
            S.cur_mask[i] = (uint16_t)((atomicAnd(&S.st[s], 0xFFFFu) >> 16) & ((1u << U) - 1));
        }
        wave_sync();
        if (lane == 0) S.n_nxt = 0;
        wave_sync();
        for (uint32_t base = 0; base < cnt; base += 64) {
            uint32_t k = cnt - base < 64u ? cnt - base : 64u;
            bool have = (uint32_t)lane < k;
            uint32_t v = 0, m = 0;
            if (have) {
                v = S.key[S.cur_slot[base + lane]];
                m = S.cur_mask[base + lane];
            }
            wave_expand<U, HLOG>(g, S, k, have, v, m, has_kids, flag_word, shift, lane, rows, edges);
        }
    }
    if (S.spill) {
        if (lane == 0) {
            spill_out[atomicAdd(spill_count, 1u)] = (uint32_t)unit;
            atomicAnd((unsigned long long *)flag_word, ~unit_bits);
        }
        return;
    }
    // pull: 64 / U lanes per request
    constexpr int LPC = 64 / U;
    const int j = lane / LPC, l = lane % LPC;
    bool ok = false;
    {
        uint32_t rr = S.root[j], t = S.target[j];
        if (rr != KETOGPU_NODE_NONE) {
            uint64_t b = g.rev_off[t], e = g.rev_off[t + 1];
            if (l == 0) rows++;
            for (uint64_t p = b + l; p < e && !ok; p += LPC) {
                uint32_t v = g.rev_col[p];
                rev++;
                if (v == rr) {
                    ok = true;
                } else if (v < g.Ni) {
                    uint32_t h = wslot<U, HLOG>(v);
                    for (int q = 0; q < H; q++, h = (h + 1) & (H - 1)) {
                        uint32_t kv = S.key[h];
                        if (kv == v) {
                            ok = (S.st[h] >> j) & 1u;
                            break;
                        }
                        if (kv == kEmpty) break;
                    }
                }
            }
        }
    }
    uint64_t bal = __ballot(ok);
    // per-wave statistics
    for (int s = 32; s; s >>= 1) {
        rows += __shfl_down(rows, s, 64);
        edges += __shfl_down(edges, s, 64);
        rev += __shfl_down(rev, s, 64);
    }
    if (lane == 0) {
        uint32_t res = 0;
        const uint64_t lm = LPC == 64 ? ~0ull : ((1ull << LPC) - 1);
        for (int q = 0; q < U; q++)
            if ((bal >> (q * LPC)) & lm) res |= 1u << q;
        if (res) atomicOr((unsigned long long *)&allowed[c0 >> 6], (unsigned long long)res << shift);
        atomicAdd(&stat_slot(stats)[0], (unsigned long long)rows);
        atomicAdd(&stat_slot(stats)[1], (unsigned long long)edges);
        atomicAdd(&stat_slot(stats)[2], (unsigned long long)rev);
    }
}

// requests of the final spill list (single requests) -> a dense batch for the global path
__global__ __launch_bounds__(kBlock) void spill_gather_kernel(const uint32_t *ids, uint64_t cnt, const uint32_t *roots,
                                                              const uint32_t *targets, uint64_t n, uint32_t *sr,
                                                              uint32_t *stt) {
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= cnt) return;
    uint64_t c = ids[i];
    sr[i] = c < n ? roots[c] : KETOGPU_NODE_NONE;
    stt[i] = c < n ? targets[c] : KETOGPU_NODE_NONE;
}

__global__ __launch_bounds__(kBlock) void spill_scatter_kernel(const uint32_t *ids, uint64_t cnt, const uint64_t *sa,
                                                               const uint64_t *sf, uint64_t *allowed, uint64_t *flags) {
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= cnt) return;
    uint64_t c = ids[i];
    unsigned long long bit = 1ull << (c & 63);
    if ((sa[i >> 6] >> (i & 63)) & 1ull) atomicOr((unsigned long long *)&allowed[c >> 6], bit);
    if ((sf[i >> 6] >> (i & 63)) & 1ull) atomicOr((unsigned long long *)&flags[c >> 6], bit);
}

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

#define HIP_CHECK(x)                                                                                   \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess)                                                                          \
            throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e));              \
    } while (0)

// every launch is checked: a failed launch must fail its call, not a later one
#define KLAUNCH(...)                                 \
    do {                                             \
        hipLaunchKernelGGL(__VA_ARGS__);             \
        HIP_CHECK(hipGetLastError());                \
    } while (0)

template <class T>
T *dalloc(size_t n) {
    void *p = nullptr;
    if (!n) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw Error(KETOGPU_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return (T *)p;
}

template <class T>
T *dupload(const std::vector<T> &v) {
    T *p = dalloc<T>(v.size());
    if (!v.empty()) HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

}  // namespace

// ------------------------------------------------ two-tier mode: launches (tier.hpp)
namespace ketogpu {
namespace tier {

static_assert(sizeof(Rec) == sizeof(FRec), "tier::Rec is the 16-byte edge record");

int stage_units_per_cu(int stage) { return stage == 1 ? 4 : 1; }

void launch_eval(int stage, const Graph &g, const Eval &e, const uint32_t *in_list, const unsigned *in_count,
                 uint32_t *out_list, unsigned *out_count, unsigned grid, hipStream_t s) {
    const bool direct = e.bnd == nullptr;
    if (stage == 0) {
        if (!e.n) return;
        const unsigned units = (unsigned)((e.n + 15) / 16);
        if (direct)
            KLAUNCH((tier_eval_kernel<LiteShape, true>), dim3(units), dim3(64), 0, s, g, e, out_list, out_count);
        else
            KLAUNCH((tier_eval_kernel<LiteShape, false>), dim3(units), dim3(64), 0, s, g, e, out_list, out_count);
    } else if (stage == 1) {
        if (direct)
            KLAUNCH((tier_cascade_kernel<TierStage1, true>), dim3(grid), dim3(64), 0, s, g, e, in_list, in_count, out_list,
                    out_count);
        else
            KLAUNCH((tier_cascade_kernel<TierStage1, false>), dim3(grid), dim3(64), 0, s, g, e, in_list, in_count, out_list,
                    out_count);
    } else {
        if (direct)
            KLAUNCH((tier_cascade_kernel<TierStage2, true>), dim3(grid), dim3(64), 0, s, g, e, in_list, in_count, out_list,
                    out_count);
        else
            KLAUNCH((tier_cascade_kernel<TierStage2, false>), dim3(grid), dim3(64), 0, s, g, e, in_list, in_count, out_list,
                    out_count);
    }
}

static unsigned tier_grid(uint64_t n, uint64_t per, unsigned cap = 8192) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, cap));
}

void launch_query_count(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n,
                        unsigned long long *counts, unsigned long long *first_bad, uint32_t *stage, hipStream_t s) {
    if (n)
        KLAUNCH(tier_query_count_kernel, dim3(tier_grid(n, kTB * 4)), dim3(kTB), 0, s, g, roots, targets, n, counts,
                first_bad, stage);
}

void launch_query_pairs(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n, Query *out,
                        unsigned long long *first_bad, uint32_t *stage, hipStream_t s) {
    if (n) KLAUNCH(tier_pair_kernel, dim3(tier_grid(n, kTB * 4)), dim3(kTB), 0, s, g, roots, targets, n, out, first_bad, stage);
}

void launch_query_scatter(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n,
                          unsigned long long *cursor, Query *out, hipStream_t s) {
    if (n) KLAUNCH(tier_query_scatter_kernel, dim3(tier_grid(n, kTB)), dim3(kTB), 0, s, g, roots, targets, n, cursor, out);
}

void launch_reply_lengths(const Graph &g, const Query *q, uint64_t n, uint64_t *lens, unsigned long long *bad,
                          hipStream_t s, uint64_t *srcb) {
    if (n) KLAUNCH(tier_reply_len_kernel, dim3(tier_grid(n, kTB * 4)), dim3(kTB), 0, s, g, q, n, lens, bad, srcb);
}

// the step's answers and status words straight into host-mapped memory (one launch instead
// of a copy each): bits (may be null) the caller's pinned answer words, h_* device views of
// the steps' pinned status words (total may be null)
// The status words are reset to "none" (~0) once copied: the next step needs no memset.
__global__ __launch_bounds__(kTB) void tier_emit_kernel(const uint64_t *allowed, uint64_t words, uint64_t *bits,
                                                        unsigned long long *status, const uint64_t *total,
                                                        unsigned long long *h_status, uint64_t *h_total) {
    for (uint64_t i = (uint64_t)blockIdx.x * kTB + threadIdx.x; i < words; i += (uint64_t)gridDim.x * kTB)
        bits[i] = allowed[i];
    if (blockIdx.x == 0 && threadIdx.x < 2) {
        h_status[threadIdx.x] = status[threadIdx.x];
        status[threadIdx.x] = ~0ull;
    }
    if (blockIdx.x == 0 && threadIdx.x == 2 && total) *h_total = *total;
}

void launch_emit(const uint64_t *allowed, uint64_t words, uint64_t *bits, unsigned long long *status,
                 const uint64_t *total, unsigned long long *h_status, uint64_t *h_total, hipStream_t s) {
    KLAUNCH(tier_emit_kernel, dim3(tier_grid(std::max<uint64_t>(words, 1), kTB, 64)), dim3(kTB), 0, s, allowed,
            bits ? words : 0, bits, status, total, h_status, h_total);
}

void launch_scan(uint64_t *v, uint64_t n, uint64_t *scratch, hipStream_t s) {
    const uint64_t nb = std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile);
    KLAUNCH(tier_scan_sums_kernel, dim3((unsigned)nb), dim3(kTB), 0, s, v, n, scratch);
    KLAUNCH(tier_scan_top_kernel, dim3(1), dim3(kTB), 0, s, scratch, nb);
    KLAUNCH(tier_scan_tiles_kernel, dim3((unsigned)nb), dim3(kTB), 0, s, v, n, scratch, nb);
}

void launch_reply_copy(const Graph &g, const Query *q, uint64_t n, const uint64_t *off, Reply *out, uint64_t cap,
                       hipStream_t s) {
    if (n) KLAUNCH(tier_reply_copy_kernel, dim3(tier_grid(n, kTB)), dim3(kTB), 0, s, g, q, n, off, out, cap);
}

void launch_seed_records(const Graph &g, const Reply *recv, uint64_t n, Rec *seed, uint4 *bnd, uint64_t nreq,
                         hipStream_t s) {
    if (n) KLAUNCH(tier_seed_kernel, dim3(tier_grid(n, kTB * kSeedPer)), dim3(kTB), 0, s, g, recv, n, seed, bnd, nreq);
}

void launch_label_reply(const Graph &g, const Query *q, uint64_t n, const uint64_t *off, const uint64_t *srcb,
                        const uint64_t *qs, uint32_t world, uint32_t *out, uint64_t cap, uint4 *bnd, uint64_t nreq,
                        hipStream_t s) {
    if (n)
        KLAUNCH(tier_label_reply_kernel, dim3(tier_grid(n, kTB)), dim3(kTB), 0, s, g, q, n, off, srcb, qs, world, out, cap,
                bnd, nreq);
}

void launch_label_lens(const uint32_t *recv, uint64_t nsent, const uint64_t *sq, const uint64_t *rp, uint32_t world,
                       uint64_t *lens, hipStream_t s) {
    if (nsent) KLAUNCH(tier_label_lens_kernel, dim3(tier_grid(nsent, kTB)), dim3(kTB), 0, s, recv, nsent, sq, rp, world, lens);
}

void launch_label_bounds(const Query *sent, uint64_t nsent, const uint64_t *sq, const uint64_t *g, uint32_t world,
                         uint4 *bnd, uint64_t nreq, uint64_t cap, hipStream_t s) {
    if (nsent)
        KLAUNCH(tier_label_bounds_kernel, dim3(tier_grid(nsent, kTB)), dim3(kTB), 0, s, sent, nsent, sq, g, world, bnd, nreq,
                cap);
}

void launch_label_eval(const Graph &g, const Eval &e, const uint32_t *recv_label, hipStream_t s) {
    if (!e.n) return;
    const unsigned units = (unsigned)((e.n + 15) / 16);
    if (recv_label)
        KLAUNCH(tier_label_kernel<false>, dim3(units), dim3(64), 0, s, g, e, recv_label);
    else
        KLAUNCH(tier_label_kernel<true>, dim3(units), dim3(64), 0, s, g, e, recv_label);
}

}  // namespace tier
}  // namespace ketogpu

// --------------------------------------------------------------------- engine
// A batch as the traversal kernels see it (device pointers)
struct Batch {
    const uint32_t *roots = nullptr, *targets = nullptr;
    uint64_t n = 0;
    uint64_t *allowed = nullptr, *flags = nullptr;
    const uint64_t *dyn_int_off = nullptr, *dyn_full_off = nullptr;
    const uint32_t *dyn_int = nullptr, *dyn_full = nullptr, *dyn_amb = nullptr;
    bool has_dyn = false;
};

// host arrays of a batch that check_host brings in chunk by chunk; mapped: pinned memory
// the device reads directly (load_kernel), else DMA copies + validate_kernel
struct HostSrc {
    const uint32_t *roots, *targets;
    bool mapped;
};

struct ketogpu_queries {
    uint64_t n = 0;
    uint32_t *d_roots = nullptr, *d_targets = nullptr;
    uint64_t *d_allowed = nullptr, *d_flags = nullptr;
    // dynamic roots of this batch
    uint64_t *d_dyn_int_off = nullptr, *d_dyn_full_off = nullptr;
    uint32_t *d_dyn_int = nullptr, *d_dyn_full = nullptr, *d_dyn_amb = nullptr;
    bool has_dyn = false;
    // the flag words are all zero (the last run on this batch was a plan-label call that
    // wrote none): with the engine's label_clean, the next such call skips the clear
    bool flags_zero = false;
    // the end of this batch's last call queued without a wait (ketogpu_queries_run_async):
    // its download waits for that call alone
    hipEvent_t done_ev = nullptr;
    bool pending = false;
    Batch batch() const {
        Batch b;
        b.roots = d_roots;
        b.targets = d_targets;
        b.n = n;
        b.allowed = d_allowed;
        b.flags = d_flags;
        b.dyn_int_off = d_dyn_int_off;
        b.dyn_full_off = d_dyn_full_off;
        b.dyn_int = d_dyn_int;
        b.dyn_full = d_dyn_full;
        b.dyn_amb = d_dyn_amb;
        b.has_dyn = has_dyn;
        return b;
    }
    ~ketogpu_queries() {
        for (void *p : {(void *)d_roots, (void *)d_targets, (void *)d_allowed, (void *)d_flags, (void *)d_dyn_int_off,
                        (void *)d_dyn_full_off, (void *)d_dyn_int, (void *)d_dyn_full, (void *)d_dyn_amb})
            if (p) (void)hipFree(p);
        if (done_ev) (void)hipEventDestroy(done_ev);
    }
};

// pinned buffers handed out by ketogpu_host_alloc: base -> (bytes, the view of every
// device that has read it; filled on first use with hipHostGetDevicePointer on that device)
struct PinnedRange {
    size_t bytes;
    std::map<int, uintptr_t> dev;  // device -> its view (0: the device cannot map it)
};
static std::mutex g_pinned_mu;
static std::map<uintptr_t, PinnedRange> g_pinned;

namespace ketogpu {
// `device`'s view of host memory it can read in place (pinned: ketogpu_host_alloc /
// hipHostMalloc / hipHostRegister; or device memory of `device`), else nullptr (the
// caller has made `device` current)
// (pageable memory goes through DMA copies).
const void *host_view(const void *p, int device, bool query, bool *is_device) {
    if (is_device) *is_device = false;
    if (!p) return nullptr;
    {  // buffers of ketogpu_host_alloc (portable + mapped): the view of THIS device,
       // known without a runtime query (~10 us per call) after its first use here
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        auto it = g_pinned.upper_bound((uintptr_t)p);
        if (it != g_pinned.begin()) {
            --it;
            const uintptr_t off = (uintptr_t)p - it->first;
            if (off < it->second.bytes) {
                auto d = it->second.dev.find(device);
                if (d == it->second.dev.end()) {
                    void *v = nullptr;  // the caller has made `device` current
                    if (hipHostGetDevicePointer(&v, (void *)it->first, 0) != hipSuccess) {
                        (void)hipGetLastError();
                        v = nullptr;
                    }
                    d = it->second.dev.emplace(device, (uintptr_t)v).first;
                }
                if (d->second) return (const void *)(d->second + off);
                return nullptr;  // not mappable here: DMA path
            }
        }
    }
    if (!query) return nullptr;
    hipPointerAttribute_t at{};
    const hipError_t e = hipPointerGetAttributes(&at, p);
    static const bool dbg = getenv("KETOGPU_DEBUG_PTR") != nullptr;
    if (dbg)
        fprintf(stderr, "[ptr] %p: err %d type %d device %d devptr %p hostptr %p managed %d flags %u\n", p, (int)e,
                (int)at.type, at.device, at.devicePointer, at.hostPointer, (int)at.isManaged, at.allocationFlags);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the query's error
        return nullptr;
    }
    if (!at.devicePointer) return nullptr;
    if (at.type == hipMemoryTypeDevice && at.device != device) return nullptr;
    if (is_device) *is_device = at.type == hipMemoryTypeDevice;
    if (at.type != hipMemoryTypeHost && at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeUnified &&
        at.type != hipMemoryTypeManaged)
        return nullptr;
    // the attributes describe the allocation: offset the device view like p
    const char *host = at.hostPointer ? (const char *)at.hostPointer : (const char *)at.devicePointer;
    const char *dev = (const char *)at.devicePointer + ((const char *)p - host);
    return (const void *)dev;
}
}  // namespace ketogpu

struct ketogpu_engine {
    const Snapshot *snap = nullptr;
    std::shared_ptr<Snapshot::ReaderLink> snap_link;  // cleared when the snapshot is freed first
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevGraph g{};
    DevState st{};
    const uint32_t *has_kids = nullptr;  // bitmap over Ni: interior node with interior successors
    uint64_t Wmax = 0;
    uint64_t *h_ctr = nullptr;  // pinned
    unsigned long long *d_hctr = nullptr;  // its device view (kernels write results there)
    std::vector<void *> owned;
    ketogpu_run_stats last{};
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    bool use_units = true;
    int wave_u = 8;
    bool use_v2 = true;
    bool use_bidi = true;
    bool use_lite = false;     // plan "lite" available (lite_kernel)
    // plan "core" (lite_kernel<CL>): lite over record arrays of its own with closure rows
    // (core_index.hpp); KETOGPU_CLOSURE="forward cap,backward cap" (0,0: the core layout
    // without closure rows)
    bool use_core = false;
    const FRec *core_rec[2] = {nullptr, nullptr};
    uint64_t core_blk[2] = {0, 0};
    uint32_t core_blk_log[2] = {0, 0}, core_block[2] = {0, 0};  // KETOGPU_CORE_BLOCKS="forward,backward" records
    uint64_t core_overflow[2] = {0, 0};
    uint32_t closure_cap[2] = {64, 64};
    // plan "label" (label_kernel): 2-hop reachability labels (labels.hpp), built at engine
    // creation; when they are, plan core and the hub index are not built (nothing would use
    // them: every request but wildcard roots is one intersection)
    bool use_label = false;
    LabelGraph lgraph{};
    // rest and full lists: kLabelSets sets each of kRestShards counters, one cache line each;
    // call k uses set k mod kLabelSets and clears set (k + kPipe) mod kLabelSets for call
    // k + kPipe — the next call on the same stream when pipelined calls rotate over kPipe
    // streams (ketogpu_queries_run_async), so a call's dense pass may still read its counters
    // while later calls' first stages run
    // streams pipelined calls rotate over (ketogpu_queries_run_async).  Two: with four, the
    // calls' first stages share the GPU fairly, end together and leave their dense passes to
    // run together with no first stage beside them (0.0754 vs 0.0614 ms per config #2 call,
    // profiles/r06/pipe/)
    static constexpr unsigned kPipe = 2;
    static constexpr unsigned kLabelSets = 2 * kPipe;
    unsigned int *rest_counts = nullptr;
    uint64_t label_calls = 0;  // selects the set
    LabelRest label_rest(uint64_t n) {    // this call's rest list over requests [0, n)
        const uint64_t units = (n + 15) / 16;
        const unsigned set = (unsigned)(label_calls % kLabelSets), next = (unsigned)((label_calls + kPipe) % kLabelSets);
        return LabelRest{spill_units, rest_counts + set * kRestShards * kRestStride,
                         rest_counts + next * kRestShards * kRestStride, 16 * ((units + kRestShards - 1) / kRestShards)};
    }
    LabelRest label_full(uint64_t n) {  // this call's list for label_full_kernel (records)
        const uint64_t units = (n + 15) / 16;
        const unsigned set = (unsigned)(label_calls % kLabelSets), next = (unsigned)((label_calls + kPipe) % kLabelSets);
        return LabelRest{nullptr, rest_counts + (kLabelSets + set) * kRestShards * kRestStride,
                         rest_counts + (kLabelSets + next) * kRestShards * kRestStride,
                         16 * ((units + kRestShards - 1) / kRestShards), full_rec + (uint64_t)set * 2 * spill_cap};
    }
    uint4 *full_rec = nullptr;  // plan label's full list per set: two records per request (kLabelSets x 2 x spill_cap)
    // KETOGPU_LABEL_FUSE=0: no lean calls (statistics, their reduction and the clear in
    // every call; A/B)
    bool fuse_reduce = [] {
        const char *e = getenv("KETOGPU_LABEL_FUSE");
        return !e || atoi(e) != 0;
    }();
    // the statistics slots and spill counters are zero (the last call was a lean one without
    // rest requests after a clear)
    bool label_clean = false;
    // this call is lean: HBM-resident plan label, timing events off, lazy rest stage
    bool lean_call = false;
    // ketogpu_queries_run_async: this call may return before the device finishes (set per
    // call); `queued`: the last call did
    bool pipelined_req = false, queued = false;
    // pipelined calls rotate over kPipe streams (by label_calls: pipe_s[0] is `stream`, the
    // others created at the first pipelined call), so one call's dense pass overlaps later
    // calls' first stages; any other work of the engine first waits for them (drain_pipe: a
    // host wait, paid only when non-pipelined work follows pipelined calls)
    hipStream_t pipe_s[kPipe] = {};
    bool pipe_used[kPipe] = {};
    // the batch each stream's last queued call ran over (compared, never dereferenced): calls
    // over the SAME batch never overlap (they write one result array), a call waits for the
    // batch's previous one (its done_ev)
    const ketogpu_queries *pipe_q[kPipe] = {};
    void drain_pipe() {
        for (unsigned k = 0; k < kPipe; k++) {
            pipe_q[k] = nullptr;
            if (k && pipe_used[k]) HIP_CHECK(hipStreamSynchronize(pipe_s[k]));
            pipe_used[k] = false;
        }
    }
    bool pipe_busy() const {
        for (unsigned k = 1; k < kPipe; k++)
            if (pipe_used[k]) return true;
        return false;
    }
    // heads marked kNoLabel by the build (the test knob) and the knob itself: with none, and
    // no head marked by a write (lab_invalid), no request of a batch without wildcard roots
    // can go to the second stage
    uint64_t label_nolabel_heads = 0;
    bool plan_auto = false;  // KETOGPU_UNITS=auto (the default)
    // lists kept in the overflow region / non-empty lists, per side (the build's histogram)
    double label_overflow_share[2] = {0, 0};
    uint32_t label_knob = 0;
    bool label_rest_free(const Batch &q) const {
        return use_label && label_nolabel_heads == 0 && label_knob == 0 && lab_invalid == 0 && !q.has_dyn;
    }
    uint64_t full_prev = 1024 * 16;  // the previous call's full-list requests (the pass's grid)
    uint32_t label_hs = 16, label_hp = 8;  // head words of S and P
    double label_coverage = 0, label_build_ms = 0, label_pll_ms = 0;
    uint64_t label_bytes = 0, label_entries = 0;
    uint64_t label_nwords[2] = {0, 0};  // words of the S and P arrays (heads + overflow)
    // writable snapshots: what label_update needs to rewrite heads in place after a write
    std::shared_ptr<const ReachLabels> lab_R;       // the 2-hop labels the heads were built from
    std::vector<uint32_t> lab_cap[2], lab_ovf[2];   // per node: entries its storage holds, overflow start / 16
    std::vector<uint64_t> lab_succ;                 // per interior node: hash of its real interior successors
    std::vector<uint8_t> lab_pinv;                  // per expandable node: P marked kNoLabel (reaches a changed row)
    uint64_t lab_invalid = 0, lab_rewritten = 0, lab_relabels = 0;
    uint32_t lab_permille = 0;
    // a head-size pair (HS, HP) as template arguments
    template <class F>
    void label_dispatch(F &&f) {
        auto hp = [&](auto hs) {
            if (label_hp == 8) f(hs, std::integral_constant<int, 8>{});
            else if (label_hp == 16) f(hs, std::integral_constant<int, 16>{});
            else if (label_hp == 32) f(hs, std::integral_constant<int, 32>{});
            else f(hs, std::integral_constant<int, 64>{});
        };
        if (label_hs == 8) hp(std::integral_constant<int, 8>{});
        else if (label_hs == 16) hp(std::integral_constant<int, 16>{});
        else if (label_hs == 32) hp(std::integral_constant<int, 32>{});
        else hp(std::integral_constant<int, 64>{});
    }
    // plan label, host batches (4 units per workgroup)
    void launch_label_host(const Batch &q, const HostSrc *src, uint64_t bunits) {
        label_dispatch([&](auto hs, auto hp) {
            KLAUNCH((label_host_kernel<decltype(hs)::value, decltype(hp)::value>), dim3((unsigned)((bunits + 3) / 4)),
                    dim3(256), 0, stream, g, lgraph, src->roots, src->targets, io->d_roots, io->d_targets, q.n,
                    q.allowed, label_rest(q.n), label_full(q.n), st.stats, d_bad);
        });
    }
    int core_shape = 2;  // KETOGPU_CORE_SHAPE: 0 = LiteShape, 1 = CoreShapeS, 2 = CoreShapeM (default: 0.195 vs 0.221 ms per 10^6 config #2 requests, profiles/r04/ab_shape)
    uint64_t closure_nodes[2] = {0, 0}, closure_entries[2] = {0, 0};
    double core_build_ms = 0;
    DevGraph gcore() const {
        DevGraph x = g;
        for (int d = 0; d < 2; d++) {
            x.blk[d] = core_blk[d];
            x.blk_log[d] = core_blk_log[d];
        }
        return x;
    }
    bool frec_needed = false;  // forward edge records built (v2, bidi, lite)
    // plan "auto" (default): the first kTrialRuns batches of >= kTrialMin requests run
    // every candidate first stage back to back (each a complete evaluation, in rotating
    // order); the engine then keeps the candidate with the smallest summed time
    static constexpr uint64_t kTrialMin = 1 << 16;
    static constexpr int kTrialRuns = 2;
    int trials_left = 0;
    struct Candidate {
        bool bidi;
        int hlog, bt, f, lf;  // bidi first-stage shape (BidiCfg)
        double ms;
        bool units = true;    // false: the global path alone (with the hub index)
        int u = 16;           // bidi: requests per first-stage unit
        int wpe = 1;          // bidi: minimum waves per SIMD of the first stage
        int lite = 0;         // bidi: plan "lite" (lite_kernel); 2: plan "core"; 3: plan "label"
    };
    std::vector<Candidate> candidates;
    // first bidi pass: table log2, threads per unit, list capacity, load limit in eighths
    // (KETOGPU_BIDI="hlog,threads,lists,load"); spilled units re-run on the spill stages
    struct BidiCfg {
        int hlog, bt, f, lf;
        int u = 16;   // requests per unit (16, or 8: half the LDS per unit)
        int wpe = 1;  // minimum waves per SIMD asked of the compiler (bidi_kernel WPE)
        int lite = 0;  // 1: plan "lite" (lite_kernel: per-unit direction, per-direction rings); 2: plan "core"; 3: "label"
        bool operator==(const BidiCfg &o) const {
            return hlog == o.hlog && bt == o.bt && f == o.f && lf == o.lf && u == o.u && wpe == o.wpe &&
                   lite == o.lite;
        }
    };
    BidiCfg bidi_cfg{9, 64, KETO_F1, 7};

    void launch_bidi(const BidiCfg &c, unsigned grid, unsigned pad, const Batch &q, const uint32_t *parents,
                     const unsigned int *in_count, uint32_t *out, unsigned int *out_count, unsigned long long *stats,
                     unsigned long long *stp, uint64_t unit0 = 0, hipStream_t stream = nullptr, bool chunked = false) {
        if (!stream) stream = this->stream;
        if (c.lite == 3) {  // plan label: 2-hop labels, plan lite for requests without
            label_dispatch([&](auto hs, auto hp) {
                KLAUNCH((label_kernel<decltype(hs)::value, decltype(hp)::value>), dim3(grid), dim3(64), pad, stream,
                        lgraph, q.roots, q.targets, q.n, q.allowed, label_rest(q.n), label_full(q.n), stats, unit0);
            });
            return;
        }
        if (c.lite == 2) {  // plan core: lite over the core record arrays
#define KETO_CORE_K(SH)                                                                                       \
    KLAUNCH((lite_kernel<SH, true>), dim3(grid), dim3(64), pad, stream, gcore(), core_rec[0], core_rec[1], q.roots, \
            q.targets, q.n, q.allowed, out, out_count, stats, unit0, stp)
            if (core_shape == 1)
                KETO_CORE_K(CoreShapeS);
            else if (core_shape == 2)
                KETO_CORE_K(CoreShapeM);
            else
                KETO_CORE_K(LiteShape);
#undef KETO_CORE_K
            return;
        }
        if (c.lite) {  // persistent spill stages never use the lite shape (parents / in_count unused)
            if (c.u == 32)
                KLAUNCH((lite_kernel<LiteShape32>), dim3(grid), dim3(64), pad, stream, g, frec, brec, q.roots,
                        q.targets, q.n, q.allowed, out, out_count, stats, unit0, stp);
            else
                KLAUNCH((lite_kernel<LiteShape>), dim3(grid), dim3(64), pad, stream, g, frec, brec, q.roots, q.targets,
                        q.n, q.allowed, out, out_count, stats, unit0, stp);
            return;
        }
        if (chunked && c == BidiCfg{9, 64, KETO_F1, 7, 16, 1}) {  // the default shape's chunk instantiation
            KLAUNCH((bidi_kernel<16, 9, KETO_F1, 64, 7, 1, 1>), dim3(grid), dim3(64), pad, stream, g, frec, brec, q.roots,
                    q.targets, q.n, q.allowed, parents, in_count, 1u, out, out_count, stats, stp, unit0);
            return;
        }
#define KETO_BIDI_U(U, HL, F, BT, LF, WPE)                                                                        \
    if (c == BidiCfg{HL, BT, F, LF, U, WPE}) {                                                                   \
        KLAUNCH((bidi_kernel<U, HL, F, BT, LF, WPE>), dim3(grid), dim3(BT), pad, stream, g, frec, brec,          \
                q.roots, q.targets, q.n, q.allowed, parents, in_count, 1u, out, out_count, stats, stp, unit0);   \
        return;                                                                                                  \
    }
#define KETO_BIDI(HL, F, BT, LF) KETO_BIDI_U(16, HL, F, BT, LF, 1)
        KETO_BIDI(11, 384, 256, 6)
        KETO_BIDI(10, 256, 256, 6)
        KETO_BIDI(10, 256, 64, 6)
        KETO_BIDI(10, 256, 64, 7)
        KETO_BIDI(9, 192, 64, 6)
        KETO_BIDI(9, 128, 64, 6)
        KETO_BIDI(9, 192, 64, 7)
        KETO_BIDI(9, 128, 64, 7)
#if KETO_F1 != 128
        KETO_BIDI(9, KETO_F1, 64, 7)
#endif
        KETO_BIDI(9, 64, 64, 7)
        KETO_BIDI(9, 96, 64, 7)
        KETO_BIDI(8, 128, 64, 7)
        KETO_BIDI(8, 96, 64, 7)
        KETO_BIDI(8, 128, 64, 6)
        KETO_BIDI_U(8, 8, 64, 64, 7, 1)
        KETO_BIDI_U(8, 8, 64, 64, 7, 6)
        KETO_BIDI_U(8, 8, 64, 64, 7, 8)
#undef KETO_BIDI
#undef KETO_BIDI_U
        throw Error(KETOGPU_EINVAL, "KETOGPU_BIDI: unsupported configuration");
    }
    // spill stages after the first bidi pass: U requests per unit, persistent grid
    struct SpillStage {
        int u;      // requests per unit (16, 4 or 1)
        char kind;  // 'w' 2048-slot 16-request table (4 waves), 'h' 1024-slot 16-request (one wave),
                    // 'q' 4096-slot 4-request (4 waves), 'r' 2048-slot 4-request (one wave),
                    // 's' 8192-slot single request (4 waves, one workgroup per CU)
    };
    // KETOGPU_CASCADE; w -> q -> s measured best on configs #2-#4 (profiles/r01/tune_cascades.txt)
    std::vector<SpillStage> cascade{{16, 'w'}, {4, 'q'}, {1, 's'}};

    // Spill stages are persistent (grid-stride over the previous stage's spilled units, a
    // count only the device knows when they launch).  Their grid follows the units the
    // stage had in the previous run (x2, at least 32 workgroups, at most the stage's full
    // grid): an empty stage of 1024 workgroups still cost ~18 us per call on config #2,
    // where one unit in 60k spills; a grid that is too small for one run only slows it.
    uint64_t stage_prev[8] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    uint64_t u2_prev[2] = {~0ull, ~0ull};  // the unit2 cascade's last units per stage
    static unsigned stage_grid(uint64_t prev, unsigned full) {
        if (prev >= full) return full;
        unsigned g = 32;
        while (g < full && g < 2 * prev) g <<= 1;
        return std::min(g, full);
    }
    void launch_stage(const SpillStage &sg, const Batch &q, const uint32_t *in, const unsigned int *in_count,
                      uint32_t fan, uint32_t *out, unsigned int *out_count, unsigned long long *stats, uint64_t prev) {
        switch (sg.kind) {
        case 'w':
            KLAUNCH((bidi_kernel<16, 11, 384, 256, 6>), dim3(stage_grid(prev, 1024)), dim3(256), 0, stream, g, frec,
                    brec, q.roots, q.targets, q.n, q.allowed, in, in_count, fan, out, out_count, stats, nullptr, 0);
            return;
        case 'q':
            KLAUNCH((bidi_kernel<4, 12, 512, 256, 7>), dim3(stage_grid(prev, 512)), dim3(256), 0, stream, g, frec,
                    brec, q.roots, q.targets, q.n, q.allowed, in, in_count, fan, out, out_count, stats, nullptr, 0);
            return;
        case 'h':
            KLAUNCH((bidi_kernel<16, 10, 256, 64, 6>), dim3(stage_grid(prev, 2048)), dim3(64), 0, stream, g, frec,
                    brec, q.roots, q.targets, q.n, q.allowed, in, in_count, fan, out, out_count, stats, nullptr, 0);
            return;
        case 'r':
            KLAUNCH((bidi_kernel<4, 11, 256, 64, 7>), dim3(stage_grid(prev, 1280)), dim3(64), 0, stream, g, frec,
                    brec, q.roots, q.targets, q.n, q.allowed, in, in_count, fan, out, out_count, stats, nullptr, 0);
            return;
        case 'L':  // plan label's second stage: plan lite over the listed requests (in: request indices)
            KLAUNCH((label_rest_kernel<TierStage1>), dim3(stage_grid(prev / 16 + 1, 256 * 4)), dim3(64), 0, stream, g,
                    frec, brec, q.roots, q.targets, q.allowed, label_rest(q.n), const_cast<unsigned int *>(in_count),
                    out, out_count, stats);
            return;
        default:
            KLAUNCH((bidi_kernel<1, 13, 1024, 256, 7>), dim3(stage_grid(prev, 256)), dim3(256), 0, stream, g, frec,
                    brec, q.roots, q.targets, q.n, q.allowed, in, in_count, fan, out, out_count, stats, nullptr, 0);
            return;
        }
    }
    const FRec *frec = nullptr;  // v2 edge records (parallel to fint_col)
    const FRec *brec = nullptr;  // v3 reverse records (parallel to rev_col)
    unsigned long long *stamps = nullptr;  // KETOGPU_STAMPS=1 diagnostic build
    std::vector<uint64_t> stat_host;
    unsigned lds_pad = 0;  // KETOGPU_LDS_PAD: extra dynamic LDS per workgroup (occupancy experiments)

    void report_stamps() {
        std::vector<unsigned long long> h((size_t)65536 * 16);
        HIP_CHECK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
        double ph[4] = {0, 0, 0, 0}, lv = 0, used = 0, lp[4] = {0, 0, 0, 0};
        std::vector<double> tot, slots, ring[2];
        for (size_t b = 0; b < 65536; b++) {
            const unsigned long long *s = &h[b * 16];
            if (s[7] != 1) continue;
            for (int k = 0; k < 4; k++) ph[k] += (double)(s[k + 1] - s[k]);
            for (int k = 0; k < 4; k++) lp[k] += (double)s[8 + k];
            lv += (double)s[5];
            used += (double)s[6];
            slots.push_back((double)s[6]);
            for (int d = 0; d < 2; d++) ring[d].push_back((double)s[12 + d]);
            tot.push_back((double)(s[4] - s[0]));
        }
        if (!slots.empty()) {  // table load and (lite) ring occupancy: p50 / p99 / max per unit
            for (auto *v : {&slots, &ring[0], &ring[1]}) std::sort(v->begin(), v->end());
            auto q = [](const std::vector<double> &v, double f) { return v[(size_t)(f * (double)(v.size() - 1))]; };
            fprintf(stderr, "[stamps] slots p50 %.0f p99 %.0f max %.0f | rings fwd p50 %.0f p99 %.0f max %.0f, "
                            "bwd p50 %.0f p99 %.0f max %.0f\n",
                    q(slots, 0.5), q(slots, 0.99), slots.back(), q(ring[0], 0.5), q(ring[0], 0.99), ring[0].back(),
                    q(ring[1], 0.5), q(ring[1], 0.99), ring[1].back());
        }
        if (tot.empty()) return;
        std::sort(tot.begin(), tot.end());
        double n = (double)tot.size();
        fprintf(stderr,
                "[stamps] units %zu  cycles/unit: init %.0f seed %.0f levels %.0f pull %.0f | total p50 %.0f p90 %.0f "
                "p99 %.0f max %.0f | levels %.2f slots %.0f\n",
                tot.size(), ph[0] / n, ph[1] / n, ph[2] / n, ph[3] / n, tot[tot.size() / 2], tot[tot.size() * 9 / 10],
                tot[tot.size() * 99 / 100], tot.back(), lv / n, used / n);
        if (lp[0] + lp[1] + lp[2] + lp[3] > 0)
            fprintf(stderr, "[stamps] bidi level phases per unit: select %.0f (unused %.0f %.0f) expand %.0f\n",
                    lp[0] / n, lp[1] / n, lp[2] / n, lp[3] / n);
        HIP_CHECK(hipMemset(stamps, 0, h.size() * 8));
    }
    // spill batch buffers (grown on demand)
    uint64_t spill_cap = 0;
    uint32_t *spill_units = nullptr, *spill_roots = nullptr, *spill_targets = nullptr;
    uint64_t *spill_allowed = nullptr, *spill_flags = nullptr;
    unsigned int *spill_count = nullptr;

    bool cascade_log = getenv("KETOGPU_CASCADE_LOG") != nullptr;  // per-stage spill counts on stderr
    // hub index (choose_hubs / build_hubs): hubs are the interior nodes with the most
    // interior successors; a search stops at a hub and the pull consults its closure
    uint32_t n_hubs = 0, hub_words = 0;
    uint64_t *hub_mask = nullptr;
    double hub_build_ms = 0;
    hipEvent_t unit_end = nullptr;  // last event of the bidi cascade (already complete after its sync)
    // host-to-host batches (check_host): persistent request/result buffers in HBM, a copy
    // stream for the chunked request upload and a second compute stream
    ketogpu_queries *io = nullptr;
    uint64_t io_cap = 0;
    hipStream_t copy_stream = nullptr, stream2 = nullptr;
    unsigned long long *d_bad = nullptr;  // smallest request index with an id outside the snapshot
    uint64_t pipe_chunk = 1 << 18;        // requests per pipelined chunk (KETOGPU_PIPE_CHUNK)
    // pinned requests read in place by one first-stage launch (bidi_host_kernel);
    // KETOGPU_PIPE_MODE=chunks restores the chunk pipeline (load_kernel + a launch per chunk)
    bool pipe_direct = true;
    // units per workgroup of the host-batch first stage (KETOGPU_HOST_UNITS: 1, 2 or 4; 0 = the
    // plan's: 4 for plan label — its units are short, so its PCIe reads bound the launch and
    // wider ones pay (0.172 vs 0.204 ms per 10^6 requests, profiles/r04/ab_label2..5) — else 2)
    int host_units = 0;
    bool light_events = true;           // timing events only around the whole call (host and device batches)
    hipEvent_t light_begin = nullptr;   // that call's begin event (run_once -> run_units)
    uint64_t *h_res = nullptr;            // pinned: a run's result words, flag words, verdict
    EmitReq emit_req;                     // host batch: emit launched with the statistics reduction
    unsigned long long *clear_bad = nullptr;  // host batch: d_bad reset by the run's clear launch
    uint64_t res_cap = 0;

    hipEvent_t ev() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }

    // Writable snapshots (snapshot_write.cpp): replay the device rows patched since the last
    // sync — each row's entries and its edge records, recomputed from the host rows (records
    // point at rows whose position and capacity never change between rebuilds).  One
    // upload of the packed rows and one scatter launch; called under the snapshot's shared
    // lock before every traversal.
    uint64_t synced_version = 0;
    uint64_t patch_pos = 0;  // absolute position in the snapshot's patch log
    // what edge records carry about the node they point at: its forward row's interior
    // successors and its reverse row's interior predecessors.  In a writable layout only the
    // real entries count (they come first; the free slots after them are never read through
    // a record), so leaf groups stay dead ends and placeholders never become pending.
    static uint32_t fdeg(const Snapshot &s, uint32_t u) {
        if (!s.writable) return (uint32_t)(s.fint_off[u + 1] - s.fint_off[u]);
        const uint32_t *b = s.fint_col.data() + s.fint_off[u], *e = s.fint_col.data() + s.fint_off[u + 1];
        return (uint32_t)(std::lower_bound(b, e, s.Df) - b);
    }
    static uint32_t ideg(const Snapshot &s, uint32_t v) {
        const uint32_t *b = s.rev_col.data() + s.rev_off[v], *e = s.rev_col.data() + s.rev_off[v + 1];
        return (uint32_t)(std::lower_bound(b, e, s.writable ? s.Dbi : s.Ni) - b);
    }
    uint64_t sync() {
        const Snapshot &s = *snap;
        // every entry point syncs first, and its work orders after the queued calls — except a
        // pipelined call with nothing to apply (its own stream and counter set order it)
        if (!pipelined_req || (bg && bg->done.load(std::memory_order_acquire)) ||
            (s.writable && synced_version != s.version))
            drain_pipe();
        if (bg && bg->done.load(std::memory_order_acquire)) finish_relabel();  // (its rows are the synced ones)
        if (!s.writable || synced_version == s.version) return 0;
        HIP_CHECK(hipSetDevice(device));
        std::vector<uint32_t> fr, rr;
        for (uint64_t i = patch_pos; i < s.patch_end(); i++) {
            const Snapshot::Patch &pt = s.patches[i - s.patch_base];
            (pt.rev ? rr : fr).push_back(pt.node);
        }
        for (auto *v : {&fr, &rr}) {
            std::sort(v->begin(), v->end());
            v->erase(std::unique(v->begin(), v->end()), v->end());
        }
        std::vector<uint64_t> seg;  // (destination, source, length, which) per row
        std::vector<uint32_t> cols;
        std::vector<FRec> recs;
        for (uint32_t v : fr) {
            const uint64_t b = s.fint_off[v], e = s.fint_off[v + 1];
            seg.insert(seg.end(), {b, (uint64_t)cols.size(), e - b, 0});
            for (uint64_t k = b; k < e; k++) {
                const uint32_t u = s.fint_col[k];
                cols.push_back(u);
                recs.push_back(FRec{u, fdeg(s, u), (uint32_t)s.fint_off[u], 0});
            }
        }
        for (uint32_t v : rr) {
            const uint64_t b = s.rev_off[v], e = s.rev_off[v + 1];
            seg.insert(seg.end(), {b, (uint64_t)cols.size(), e - b, 1});
            for (uint64_t k = b; k < e; k++) {
                const uint32_t u = s.rev_col[k];
                cols.push_back(u);
                recs.push_back(u < s.Ni ? FRec{u, ideg(s, u), (uint32_t)s.rev_off[u], 0} : FRec{u, 0, 0, 0});
            }
        }
        const uint64_t nseg = seg.size() / 4;
        if (nseg && !cols.empty()) {
            uint64_t *d_seg = dupload(seg);
            uint32_t *d_cols = dupload(cols);
            FRec *d_recs = dupload(recs);
            KLAUNCH(patch_rows_kernel, dim3((unsigned)std::min<uint64_t>(nseg, 65535)), dim3(256), 0, stream, d_seg,
                    nseg, d_cols, d_recs, const_cast<uint32_t *>(g.fint_col), const_cast<FRec *>(frec),
                    const_cast<uint32_t *>(g.rev_col), const_cast<FRec *>(brec));
            HIP_CHECK(hipStreamSynchronize(stream));
            for (void *p : {(void *)d_seg, (void *)d_cols, (void *)d_recs}) (void)hipFree(p);
        }
        g.N = s.N;
        if (use_label) label_update(fr, rr);
        patch_pos = s.patch_end();
        s.reader_at(this, patch_pos);
        synced_version = s.version;
        return nseg;
    }

    // hash of an interior node's real interior successors (writable rows: those below Dbi)
    static uint64_t succ_hash(const Snapshot &s, uint32_t v) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (uint64_t k = s.fint_off[v]; k < s.fint_off[v + 1]; k++) {
            const uint32_t u = s.fint_col[k];
            if (u >= s.Dbi) break;  // the free slots (sorted last)
            h = mix64(h ^ (u + 0x5851F42D4C957F2Dull));
        }
        return h;
    }

    // Plan label after an in-place write (writable snapshots), exact without a rebuild:
    //  * a changed reverse row rev(t): S(t) recomputed from the current row and the labels'
    //    Lin (the interior graph's labels are unchanged unless an interior row changed);
    //  * a changed forward row of a non-interior node r: P(r) recomputed;
    //  * an interior node v whose real interior successors changed (a nesting edge added or
    //    removed): every expandable node that reaches v (backward over the current rows) gets
    //    P = no label, so requests from those roots go to the second stage (plan lite over the
    //    live device rows).  Exact: a request whose answer the change can alter has a root
    //    that reaches a changed node; for any other root r, r's reachable region is unchanged
    //    and so is every landmark w in it, so Lout(r) meets Lin(v) iff r ->* v as before.
    //    Marks are kept (a later edge into a marked node marks its new predecessor too).
    //  * a list that outgrows its node's storage: no label (second stage) until the relabel.
    // When the marked heads pass KETOGPU_LABEL_RELABEL_PERMILLE of the P nodes (default 20),
    // the labels are rebuilt from the current rows (relabel).
    void label_update(const std::vector<uint32_t> &fr, const std::vector<uint32_t> &rr) {
        const Snapshot &s = *snap;
        if (!s.writable || !lab_R) return;
        if (bg) {  // a background relabel in flight: its swap re-applies every row changed since its copy
            bg->fr.insert(bg->fr.end(), fr.begin(), fr.end());
            bg->rr.insert(bg->rr.end(), rr.begin(), rr.end());
        }
        const ReachLabels &R = *lab_R;
        std::vector<uint32_t> seeds;
        for (uint32_t v : fr)
            if (v < s.Ni && v != s.Df && v != s.Dbi) {
                const uint64_t h = succ_hash(s, v);
                if (h != lab_succ[v]) seeds.push_back(v), lab_succ[v] = h;
            }
        std::vector<uint32_t> marked;  // P heads newly marked no label
        for (size_t h = 0; h < seeds.size(); h++) {  // seeds grows: a backward search
            const uint32_t y = seeds[h];
            if (lab_pinv[y]) continue;
            lab_pinv[y] = 1;
            marked.push_back(y);
            for (uint64_t k = s.rev_off[y]; k < s.rev_off[y + 1]; k++) {
                const uint32_t p = s.rev_col[k];
                if (p != s.Dbi && p != s.Dbo && p < s.Nx && !lab_pinv[p]) seeds.push_back(p);
            }
        }
        std::vector<uint32_t> rec[2];
        std::vector<uint64_t> roff[2];
        std::vector<uint32_t> l;
        auto emit = [&](int side, uint32_t x, bool nolabel, uint64_t mask) {
            const uint32_t h = side == 0 ? label_hs : label_hp, c = (uint32_t)l.size();
            const bool fits = !nolabel && c <= lab_cap[side][x];
            std::vector<uint32_t> &r = rec[side];
            roff[side].push_back(r.size());
            r.push_back(x);
            r.push_back(fits ? c : 0u);  // entries the patch copies to the overflow region
            const size_t hd = r.size();
            r.resize(hd + h, 0xFFFFFFFFu);
            if (!fits) {
                r[hd] = kNoLabel, r[hd + 1] = r[hd + 2] = r[hd + 3] = 0;
                lab_invalid += !nolabel || side == 1;
                return;
            }
            const bool inl = c <= h - kHeadFixed;
            r[hd] = c;
            r[hd + 1] = inl ? 0u : lab_ovf[side][x];
            r[hd + 2] = (uint32_t)mask;
            r[hd + 3] = (uint32_t)(mask >> 32);
            std::copy(l.begin(), l.begin() + std::min<size_t>(c, h - kHeadFixed), r.begin() + (ptrdiff_t)(hd + kHeadFixed));
            if (!inl) r.insert(r.end(), l.begin(), l.end());
            lab_rewritten++;
        };
        uint64_t mask = 0;
        for (uint32_t t : rr) {
            if (t >= lab_cap[0].size()) continue;
            label_list(s, R, false, t, l, mask);
            emit(0, t, !l.empty() && label_nolabel(t, lab_permille), mask);
        }
        for (uint32_t x : marked) {
            l.clear();
            emit(1, x, true, 0);
        }
        for (uint32_t r : fr) {
            if (r < s.Ni || r >= s.Nx || lab_pinv[r]) continue;
            bool stale = false;  // an entry that reaches a changed node: its Lout may be stale
            for (uint64_t k = s.fint_off[r]; k < s.fint_off[r + 1] && !stale; k++) {
                const uint32_t c = s.fint_col[k];
                stale = c != s.Df && lab_pinv[c];
            }
            if (stale) {
                lab_pinv[r] = 1;
                l.clear();
                emit(1, r, true, 0);
                continue;
            }
            label_list(s, R, true, r, l, mask);
            emit(1, r, false, mask);
        }
        for (int side = 0; side < 2; side++) {
            if (roff[side].empty()) continue;
            uint32_t *drec = dupload(rec[side]);
            uint64_t *droff = dupload(roff[side]);
            KLAUNCH(label_patch_kernel, dim3((unsigned)std::min<size_t>(roff[side].size(), 4096)), dim3(64), 0, stream,
                    drec, droff, (uint32_t)roff[side].size(), const_cast<uint32_t *>(side == 0 ? lgraph.S : lgraph.P),
                    side == 0 ? label_hs : label_hp);
            HIP_CHECK(hipStreamSynchronize(stream));
            (void)hipFree(drec);
            (void)hipFree(droff);
        }
        uint64_t limit = 20;
        if (const char *e = getenv("KETOGPU_LABEL_RELABEL_PERMILLE")) limit = strtoull(e, nullptr, 10);
        if (!bg && lab_invalid * 1000 > limit * std::max<uint64_t>(s.Nx, 1)) {
            static const bool inline_relabel = getenv("KETOGPU_LABEL_RELABEL_SYNC") != nullptr;
            if (inline_relabel)
                relabel();
            else
                start_relabel();
        }
    }

    // Background relabel: the 2-hop labels of the current interior graph are built on a host
    // thread from a copy of it (copy_interior), so the write that crossed the threshold — and
    // the writes after it — return without waiting; until the swap, marked roots keep going
    // to the second stage over the live rows.  The swap (at the first engine sync after the
    // build finished, finish_relabel) builds the head arrays from the new labels over the
    // current rows and then applies label_update to every row changed since the copy,
    // against the interior successor hashes of the copy: exact by label_update's own argument
    // (the labels are those of the copied interior graph; a root reaching an interior row
    // changed since is marked).  KETOGPU_LABEL_RELABEL_SYNC=1: the relabel inline (A/B).
    struct BgRelabel {
        std::thread th;
        std::atomic<bool> done{false};
        std::shared_ptr<ReachLabels> R;   // the new labels (null: the build failed)
        std::vector<uint64_t> succ;       // interior successor hashes of the copy
        std::vector<uint32_t> fr, rr;     // rows changed since the copy
        std::string error;
    };
    std::unique_ptr<BgRelabel> bg;
    uint64_t lab_bg_started = 0;
    void start_relabel() {
        const Snapshot &s = *snap;
        auto b = std::make_unique<BgRelabel>();
        auto c = std::make_shared<InteriorCsr>();
        copy_interior(s, *c);  // (under the caller's snapshot lock)
        b->succ.resize(s.Ni);
        for (uint32_t v = 0; v < s.Ni; v++) b->succ[v] = succ_hash(s, v);
        const uint64_t version = s.version;
        BgRelabel *bp = b.get();
        bp->th = std::thread([bp, c, version] {
            try {
                auto R = std::make_shared<ReachLabels>();
                build_reach_labels_csr(c->n, c->f_off.data(), c->f_col.data(), c->b_off.data(), c->b_col.data(), *R);
                R->version = version;
                bp->R = std::move(R);
            } catch (const std::exception &e) {
                bp->error = e.what();
            }
            bp->done.store(true, std::memory_order_release);
        });
        bg = std::move(b);
        lab_bg_started++;
    }
    void finish_relabel() {
        std::unique_ptr<BgRelabel> b = std::move(bg);
        b->th.join();
        if (!b->R) {  // the build failed: the relabel inline (it reports its own failure)
            fprintf(stderr, "[ketogpu] background relabel failed (%s): relabelling inline\n", b->error.c_str());
            relabel();
            return;
        }
        uint32_t *A[2] = {const_cast<uint32_t *>(lgraph.S), const_cast<uint32_t *>(lgraph.P)};
        release_label(A);
        lgraph = LabelGraph{nullptr, nullptr, 0};
        lab_R.reset();
        use_label = true;
        build_label(*snap, b->R);
        if (!use_label || !lab_R) return;  // (the heads did not fit: plan lite, as build_label decided)
        lab_succ = std::move(b->succ);  // the interior graph the labels describe
        for (auto *v : {&b->fr, &b->rr}) {
            std::sort(v->begin(), v->end());
            v->erase(std::unique(v->begin(), v->end()), v->end());
        }
        label_update(b->fr, b->rr);
        lab_relabels++;
    }

    // the labels rebuilt from the current rows (the old arrays freed first)
    void relabel() {
        uint32_t *A[2] = {const_cast<uint32_t *>(lgraph.S), const_cast<uint32_t *>(lgraph.P)};
        release_label(A);
        lgraph = LabelGraph{nullptr, nullptr, 0};
        lab_R.reset();
        use_label = true;
        build_label(*snap);
        lab_relabels++;
    }

    ~ketogpu_engine() {
        if (bg && bg->th.joinable()) bg->th.join();  // (a background relabel reads only its own copy)
        if (snap_link) {
            std::lock_guard<std::mutex> lk(snap_link->mu);
            if (snap_link->snap) snap_link->snap->reader_gone(this);
        }
        // every stream of the engine drains before anything it may read or write is freed
        // (the chunk pipeline's copies run on copy_stream and its launches on stream2)
        (void)hipSetDevice(device);
        for (hipStream_t x : {stream, stream2, copy_stream})
            if (x) (void)hipStreamSynchronize(x);
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        if (wait_ev) (void)hipEventDestroy(wait_ev);
        for (unsigned k = 1; k < kPipe; k++)
            if (pipe_s[k]) {
                (void)hipStreamSynchronize(pipe_s[k]);
                (void)hipStreamDestroy(pipe_s[k]);
            }
        for (void *p : owned) (void)hipFree(p);
        for (void *p : {(void *)spill_units, (void *)spill_roots, (void *)spill_targets, (void *)spill_allowed,
                        (void *)spill_flags, (void *)full_rec})
            if (p) (void)hipFree(p);
        if (h_ctr) (void)hipHostFree(h_ctr);
        if (h_res) (void)hipHostFree(h_res);
        delete io;
        for (hipStream_t x : {copy_stream, stream2})
            if (x) (void)hipStreamDestroy(x);
        if (stream) (void)hipStreamDestroy(stream);
    }

    void init(const Snapshot &s, const ketogpu_engine_opts *o) {
        snap = &s;
        device = o ? o->device : 0;
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw Error(KETOGPU_EDEVICE, "no such HIP device");
        HIP_CHECK(hipSetDevice(device));
        HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
        if (const char *pc = getenv("KETOGPU_PIPE_CHUNK"))  // requests per chunk, rounded to 64
            pipe_chunk = std::max<uint64_t>(64, (uint64_t)atoll(pc) / 64 * 64);
        if (const char *pm = getenv("KETOGPU_PIPE_MODE")) pipe_direct = std::string(pm) != "chunks";
        if (const char *hu = getenv("KETOGPU_HOST_UNITS")) host_units = atoi(hu);
        if (const char *ea = getenv("KETOGPU_EVENTS")) light_events = std::string(ea) != "all";
        if (s.N >= kDynBase) throw Error(KETOGPU_EINVAL, "snapshot has >= 2^31 nodes");
        const char *mode = getenv("KETOGPU_PATH");  // "global": skip the LDS unit path (tests)
        use_units = !(mode && std::string(mode) == "global");
        // first LDS pass: "bidi" (default) = bidi_kernel, bidirectional search per request,
        // spills continue on the v2 cascade; "v2" = unit2_kernel, one workgroup per 16
        // requests with edge records; "b16" = unit_kernel; "w4" / "w8" / "w16" = one wave
        // per 4/8/16 requests.  Spills go on to 4-request and 1-request units, then the
        // global path.
        const char *plan = getenv("KETOGPU_UNITS");
        std::string p = plan ? plan : "auto";
        wave_u = p == "w4" ? 4 : p == "w8" ? 8 : p == "w16" ? 16 : 0;
        const bool lite_req = p == "lite" || p == "lite32" || p == "core" || p == "label" || p == "auto";
        use_v2 = p == "v2" || p == "bidi" || lite_req;
        // Edge records carry 32-bit row begins.  Plan lite reads only INTERIOR rows through
        // records (ids below Ni come first, so their begins are the smallest) and carries
        // seed rows' begins in 64 bits: it needs fint_off[Ni] and rev_off[Ni] below 2^32.
        // bidi and unit2 also keep seed begins in 32 bits: they need every row below 2^32.
        const bool small_f = s.fint_col.size() < (1ull << 32), small_r = s.rev_col.size() < (1ull << 32);
        const bool lite_ok = s.fint_off[s.Ni] < (1ull << 32) && s.rev_off[s.Ni] < (1ull << 32);
        const bool recs = use_v2 && (small_f || (lite_req && lite_ok));
        auto disabled = [&](const char *what, const char *why) {
            fprintf(stderr, "[ketogpu] plan %s disabled: %s (fint %llu, rev %llu entries; interior rows %llu / %llu)\n",
                    what, why, (unsigned long long)s.fint_col.size(), (unsigned long long)s.rev_col.size(),
                    (unsigned long long)s.fint_off[s.Ni], (unsigned long long)s.rev_off[s.Ni]);
        };
        // bidi / lite: R4 flags come from forward rows, so snapshots with ambiguous keys stay on v2
        use_lite = lite_req && use_v2 && !s.has_ambiguous && lite_ok;
        // plan core: not on writable snapshots (an in-place write would change closures)
        use_core = (p == "core" || p == "auto") && use_lite && !s.writable && getenv("KETOGPU_NO_CORE") == nullptr;
        // (labels on a writable snapshot are kept exact in place by label_update)
        use_label = (p == "label" || p == "auto") && use_lite && getenv("KETOGPU_NO_LABEL") == nullptr;
        if (const char *e = getenv("KETOGPU_CLOSURE")) sscanf(e, "%u,%u", &closure_cap[0], &closure_cap[1]);
        if (const char *e = getenv("KETOGPU_CORE_SHAPE")) core_shape = atoi(e);
        if (const char *e = getenv("KETOGPU_CORE_BLOCKS")) sscanf(e, "%u,%u", &core_block[0], &core_block[1]);
        use_bidi = (p == "bidi" || p == "auto") && use_v2 && !s.has_ambiguous && small_f && small_r;
        if (use_v2 && !small_f) {
            disabled("v2", "forward rows pass 2^32 entries (32-bit record begins)");
            use_v2 = false;
        }
        if ((p == "bidi" || p == "auto") && !s.has_ambiguous && recs && !use_bidi)
            disabled("bidi", "rows pass 2^32 entries (32-bit seed begins)");
        if (lite_req && !s.has_ambiguous && !lite_ok) disabled("lite", "interior rows pass 2^32 entries");
        frec_needed = recs && (use_v2 || use_bidi || use_lite);
        if (p == "core" && use_core) {  // forced: plan core, no trials
            use_bidi = true;
            bidi_cfg = BidiCfg{9, 64, kLiteF, 7, 16, 1, 2};
        }
        if (p == "label" && use_label) {  // forced: plan label (falls back to lite if the labels do not fit)
            use_bidi = true;
            bidi_cfg = BidiCfg{9, 64, kLiteF, 7, 16, 1, 3};
        }
        if ((p == "lite" || p == "lite32") && use_lite) {  // forced: the lite first stage, no trials
            use_bidi = true;
            bidi_cfg.lite = 1;
            bidi_cfg.hlog = p == "lite32" ? 10 : 9;
            bidi_cfg.f = p == "lite32" ? 2 * kLiteF : kLiteF;
            bidi_cfg.u = p == "lite32" ? 32 : 16;
        }
        trials_left = p == "auto" && (use_bidi || use_lite) && use_units ? kTrialRuns : 0;
        if (const char *pad = getenv("KETOGPU_LDS_PAD")) lds_pad = (unsigned)atoi(pad);
        const char *bc = getenv("KETOGPU_BIDI");  // "hlog,threads,lists,load", e.g. "9,64,192,6"
        if (bc) {
            BidiCfg c = bidi_cfg;
            if (sscanf(bc, "%d,%d,%d,%d,%d,%d", &c.hlog, &c.bt, &c.f, &c.lf, &c.u, &c.wpe) >= 1) bidi_cfg = c;
        }
        if (trials_left) {
            // candidates: the bidi shape (128-entry lists), bidi with 64-entry lists (spills
            // sooner: better where most units spill anyway, config #4), forward-only unit2
            // (chains, config #3); an explicit KETOGPU_BIDI shape replaces the two bidi ones
            // (8-request units — 5 KB of LDS, KETOGPU_BIDI=8,64,64,7,8[,wpe] — measured slower on
            // config #2: 0.48-0.53 vs 0.39 ms, profiles/r01/tune_u8.txt; not a candidate)
            const BidiCfg &c = bidi_cfg;
            if (use_bidi) {
                candidates.push_back({true, c.hlog, c.bt, c.f, c.lf, 0, true, c.u, c.wpe});
                if (!bc) candidates.push_back({true, 9, 64, 64, 7, 0});
            }
            if (use_lite) candidates.push_back({true, 9, 64, kLiteF, 7, 0, true, 16, 1, 1});  // plan "lite"
            if (use_core) candidates.push_back({true, 9, 64, kLiteF, 7, 0, true, 16, 1, 2});  // plan "core"
            if (use_v2) candidates.push_back({false, c.hlog, c.bt, c.f, c.lf, 0});
            // batches below the trial size run lite until the trials have picked a plan
            // (round 3: lite 0.284 vs bidi 0.367 ms per 10^6 config #2 requests)
            if (use_lite && !bc) bidi_cfg = BidiCfg{9, 64, kLiteF, 7, 16, 1, use_core ? 2 : 1};
            use_bidi = use_bidi || use_lite;
        }
        if (const char *cs = getenv("KETOGPU_CASCADE")) {  // spill stages, e.g. "w,q,s" (default) or "q,s"
            std::vector<SpillStage> c;
            for (const char *p = cs; *p; p++) {
                if (*p == 'w' || *p == 'h') c.push_back({16, *p});
                else if (*p == 'q' || *p == 'r') c.push_back({4, *p});
                else if (*p == 's') c.push_back({1, 's'});
            }
            if (c.empty() || c.back().kind != 's' || c.size() > 6)
                throw Error(KETOGPU_EINVAL, "KETOGPU_CASCADE: stages w|h|q|r|s ending with s, at most 6");
            cascade = c;
        }
        if (getenv("KETOGPU_STAMPS")) {
            stamps = dalloc<unsigned long long>((size_t)65536 * 16);
            owned.push_back(stamps);
            HIP_CHECK(hipMemset(stamps, 0, (size_t)65536 * 16 * 8));
        }
        auto up = [&](auto &vec) {
            auto *p = dupload(vec);
            owned.push_back((void *)p);
            return p;
        };
        g.fint_off = up(s.fint_off);
        g.fint_col = up(s.fint_col);
        g.rev_off = up(s.rev_off);
        g.rev_col = up(s.rev_col);
        g.row_amb = s.has_ambiguous ? up(s.row_amb) : nullptr;
        g.Ni = s.Ni;
        g.Nx = s.Nx;
        g.N = s.N;
        // plan label first: when its labels are built every request but wildcard roots is
        // one intersection, so neither plan core's index nor the hub index is built, and no
        // trials run (KETOGPU_UNITS=auto)
        plan_auto = p == "auto";
        if (use_label) build_label(s);
        g.both_max = kBothMax;
        g.seed_shift = 0;
        if (const char *sh = getenv("KETOGPU_TEST_BEGIN_SHIFT")) g.seed_shift = strtoull(sh, nullptr, 0);
        g.seed_max = kSeedBothMax;
        if (const char *bt = getenv("KETOGPU_BIDI_TUNE")) {  // "both,seed" (tuning runs)
            unsigned a = kBothMax, b = kSeedBothMax;
            if (sscanf(bt, "%u,%u", &a, &b) >= 1) g.both_max = a, g.seed_max = b;
        }
        {
            std::vector<uint32_t> hk(((size_t)s.Ni + 31) / 32 + 1, 0);
            for (uint32_t v = 0; v < s.Ni; v++)
                if (s.fint_off[v + 1] > s.fint_off[v]) hk[v >> 5] |= 1u << (v & 31);
            has_kids = up(hk);
        }
        choose_hubs(s);
        if (frec_needed) {
            std::vector<FRec> rec(s.fint_col.size());
            for (size_t e = 0; e < rec.size(); e++) {
                uint32_t u = s.fint_col[e];
                const uint32_t hid = hub_of_h.empty() ? KETOGPU_NODE_NONE : hub_of_h[u];
                rec[e] = FRec{u, fdeg(s, u), (uint32_t)s.fint_off[u], hid == KETOGPU_NODE_NONE ? 0u : hid + 1};
            }
            frec = up(rec);
        }
        if (use_bidi || use_lite) {
            // interior predecessors of v = the prefix of rev(v) below Ni (sorted rows)
            std::vector<uint32_t> id(s.Ni);
            for (uint32_t v = 0; v < s.Ni; v++) id[v] = ideg(s, v);
            std::vector<FRec> rec(s.rev_col.size());
            for (size_t e = 0; e < rec.size(); e++) {
                uint32_t v = s.rev_col[e];
                rec[e] = v < s.Ni ? FRec{v, id[v], (uint32_t)s.rev_off[v], 0} : FRec{v, 0, 0, 0};
            }
            brec = up(rec);
        }
        if (use_core) build_core(s);

        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        uint64_t budget = o && o->state_budget_bytes ? o->state_budget_bytes
                                                     : std::min<uint64_t>(free_b / 4, (uint64_t)64 << 30);
        budget = std::min<uint64_t>(budget, (uint64_t)free_b * 3 / 4);
        // frontier lists: 24 B per entry, touch list 8 B; vis+nxt: 16 B per (word, node)
        uint64_t lists = std::min<uint64_t>(budget / 4, (uint64_t)24 << 30);
        st.fe_cap = std::min<uint64_t>(std::max<uint64_t>(lists / 32, 1 << 16), kMaxListEntries);
        st.touch_cap = st.fe_cap;
        // per 64-request word: vis + nxt rows and the requests' hub reach bitmaps
        uint64_t per_word = 16ull * std::max<uint32_t>(s.Ni, 1) + 64ull * 8 * hub_words;
        Wmax = std::max<uint64_t>(1, (budget - std::min(budget, lists)) / per_word);
        if (o && o->max_words_per_round) Wmax = std::min<uint64_t>(Wmax, o->max_words_per_round);
        Wmax = std::min<uint64_t>(Wmax, 1u << 20);
        // a round appends each (word, node) pair at most once (plus its seeds), so a round of
        // W <= fe_cap / (Ni + 64) words never overflows the lists (no retries at any degree)
        Wmax = std::max<uint64_t>(1, std::min<uint64_t>(Wmax, st.fe_cap / ((uint64_t)s.Ni + 64)));
        size_t state = (size_t)Wmax * std::max<uint32_t>(s.Ni, 1);
        st.vis = dalloc<uint64_t>(state);
        owned.push_back(st.vis);
        st.nxt = dalloc<uint64_t>(state);
        owned.push_back(st.nxt);
        HIP_CHECK(hipMemsetAsync(st.vis, 0, state * 8, stream));
        HIP_CHECK(hipMemsetAsync(st.nxt, 0, state * 8, stream));
        st.fe_key = dalloc<uint64_t>(st.fe_cap);
        st.fe_mask = dalloc<uint64_t>(st.fe_cap);
        st.fe_pre = dalloc<uint64_t>(st.fe_cap);
        st.touch = dalloc<uint64_t>(st.touch_cap);
        for (void *p : {(void *)st.fe_key, (void *)st.fe_mask, (void *)st.fe_pre, (void *)st.touch}) owned.push_back(p);
        st.ctr = dalloc<unsigned long long>(8);
        st.overflow = dalloc<unsigned int>(4);
        st.stats = dalloc<unsigned long long>(kStatsLen);
        spill_count = (unsigned int *)(st.stats + 8 + 8 * kStatSlots + 8);
        for (void *p : {(void *)st.ctr, (void *)st.overflow, (void *)st.stats}) owned.push_back(p);  // spill_count lives in st.stats
        HIP_CHECK(hipHostMalloc((void **)&h_ctr, 64 * sizeof(uint64_t), hipHostMallocDefault));
        HIP_CHECK(hipHostGetDevicePointer((void **)&d_hctr, h_ctr, 0));
        d_bad = dalloc<unsigned long long>(1);
        owned.push_back(d_bad);
        HIP_CHECK(hipStreamSynchronize(stream));
        build_hubs(s);
    }

    // plan core's record arrays (core_index.hpp): built on the host, uploaded; the plan is
    // dropped (with a message) when they do not fit a quarter of free HBM or pass 2^32
    // core records
    void build_core(const Snapshot &s) {
        CoreIndex ci;
        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        try {  // (the record arrays' size is checked against a quarter of free HBM before allocating)
            build_core_index(s, closure_cap, core_block, ci, free_b / 4);
        } catch (const Error &e) {
            fprintf(stderr, "[ketogpu] plan core disabled: %s\n", e.what());
            drop_core();
            return;
        } catch (const std::bad_alloc &) {
            fprintf(stderr, "[ketogpu] plan core disabled: out of host memory\n");
            drop_core();
            return;
        }
        const uint64_t bytes = (ci.rec[0].size() + ci.rec[1].size()) * sizeof(CoreRec);
        if (bytes > free_b / 4) {
            fprintf(stderr, "[ketogpu] plan core disabled: %llu bytes of records, %llu free\n",
                    (unsigned long long)bytes, (unsigned long long)free_b);
            drop_core();
            return;
        }
        for (int d = 0; d < 2; d++) {
            CoreRec *p = dupload(ci.rec[d]);
            owned.push_back(p);
            core_rec[d] = reinterpret_cast<const FRec *>(p);
            core_blk[d] = ci.block_base[d];
            core_blk_log[d] = ci.block_log[d];
            core_overflow[d] = ci.overflow_rows[d];
            closure_nodes[d] = ci.closure_nodes[d];
            closure_entries[d] = ci.closure_entries[d];
        }
        core_build_ms = ci.build_ms;
        if (cascade_log)
            fprintf(stderr, "[core] closure rows: forward %llu nodes / %llu entries, backward %llu / %llu (caps %u, %u); "
                            "blocks of %u / %u records, %llu / %llu rows in overflow; %.2f GB; built in %.1f ms\n",
                    (unsigned long long)closure_nodes[0], (unsigned long long)closure_entries[0],
                    (unsigned long long)closure_nodes[1], (unsigned long long)closure_entries[1], closure_cap[0],
                    closure_cap[1], 1u << core_blk_log[0], 1u << core_blk_log[1], (unsigned long long)core_overflow[0],
                    (unsigned long long)core_overflow[1], (double)bytes / 1e9, core_build_ms);
    }
    void drop_label() {
        use_label = false;
        if (bidi_cfg.lite == 3) bidi_cfg.lite = use_core ? 2 : 1;
    }
    void drop_core() {
        use_core = false;
        candidates.erase(std::remove_if(candidates.begin(), candidates.end(), [](const Candidate &c) { return c.lite == 2; }),
                         candidates.end());
        if (bidi_cfg.lite == 2) bidi_cfg.lite = 1;
    }
    // plan label's 2-hop labels (labels.hpp, built once per snapshot on the host and shared
    // by its engines) and the head arrays, built on the device from them and the graph in
    // HBM (label_count_kernel / label_write_kernel; KETOGPU_LABEL_HOST=1: the host build,
    // uploaded).  The arrays must fit half of the HBM left after the graph and its edge
    // records (checked before they are allocated).  On success the plan is label without
    // trials, and plan core and the hub index are skipped; on failure the engine goes on as
    // if labels had not been asked for.
    void build_label(const Snapshot &s, std::shared_ptr<const ReachLabels> given = nullptr) {
        const auto t0 = std::chrono::steady_clock::now();
        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        const uint64_t records = 16ull * (s.fint_col.size() + s.rev_col.size());
        const uint64_t budget = free_b > records ? (free_b - records) / 2 : 0;
        uint32_t hs = 0, hp = 0, permille = 0;
        if (const char *e = getenv("KETOGPU_LABEL_HEADS")) sscanf(e, "%u,%u", &hs, &hp);
        if (const char *e = getenv("KETOGPU_LABEL_REST_PERMILLE")) permille = (uint32_t)std::min(1000, std::max(0, atoi(e)));
        for (uint32_t h : {hs, hp})
            if (h && h != 8 && h != 16 && h != 32 && h != 64) {
                fprintf(stderr, "[ketogpu] plan label disabled: KETOGPU_LABEL_HEADS takes 8, 16, 32 or 64 words\n");
                drop_label();
                return;
            }
        std::vector<void *> tmp;  // device temporaries of the build
        auto free_tmp = [&] {
            for (void *p : tmp) (void)hipFree(p);
            tmp.clear();
        };
        uint32_t *A[2] = {nullptr, nullptr};  // S, P
        uint32_t H[2] = {hs, hp};
        uint64_t nolabel = 0, s_entries = 0, nonempty_s = 0;
        try {
            if (getenv("KETOGPU_LABEL_HOST")) {  // the host build (A/B, and the test hook's path)
                LabelIndex li;
                build_labels(s, hs, hp, permille, budget, li);
                A[0] = dupload(li.S);
                owned.push_back(A[0]);
                A[1] = dupload(li.P);
                owned.push_back(A[1]);
                H[0] = li.hs, H[1] = li.hp;
                label_nwords[0] = li.S.size();
                label_nwords[1] = li.P.size();
                label_bytes = 4 * (li.S.size() + li.P.size());
                label_entries = li.label_entries;
                label_pll_ms = li.pll_ms;
                nolabel = li.s_nolabel;
                s_entries = li.s_entries;
            } else {
                const std::shared_ptr<const ReachLabels> R = given ? given : reach_labels_of(s);
                label_pll_ms = R->ms;
                label_entries = R->in.size() + R->out.size();
                auto up = [&](const auto &v) {
                    using T = typename std::decay_t<decltype(v)>::value_type;
                    T *p = dalloc<T>(std::max<size_t>(v.size(), 1));
                    tmp.push_back(p);
                    if (!v.empty()) HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
                    return p;
                };
                LabelDevLists D{up(R->in_off), up(R->out_off), up(R->in), up(R->out), up(R->min), up(R->mout), s.Ni,
                                {s.writable ? s.Df : NONE, s.writable ? s.Dbi : NONE, s.writable ? s.Dbo : NONE}};
                unsigned long long *ctr = dalloc<unsigned long long>(8);
                tmp.push_back(ctr);
                uint64_t used = 0;
                label_bytes = 0;
                for (int side = 0; side < 2; side++) {
                    const uint32_t n = side == 0 ? (uint32_t)label_s_nodes(s) : s.Nx;
                    uint32_t *cnt = dalloc<uint32_t>(std::max<uint32_t>(n, 1)), *off16 = dalloc<uint32_t>(std::max<uint32_t>(n, 1));
                    tmp.push_back(cnt);
                    tmp.push_back(off16);
                    uint32_t big_cap = std::max<uint32_t>(4096, n / 32);
                    if (const char *e = getenv("KETOGPU_TEST_LABEL_BIG_CAP"))  // (tests: the regrow below)
                        big_cap = std::max(1, atoi(e));
                    uint32_t *big = dalloc<uint32_t>(big_cap);
                    tmp.push_back(big);
                    HIP_CHECK(hipMemsetAsync(ctr, 0, 8 * sizeof(unsigned long long), stream));
                    const unsigned grid = (unsigned)std::min<uint64_t>(std::max<uint64_t>((n + 3) / 4, 1), 16384);
                    if (n) {
                        if (side == 0)
                            KLAUNCH(label_count_kernel<false>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, ctr, big,
                                    (unsigned int *)(ctr + 6), big_cap);
                        else
                            KLAUNCH(label_count_kernel<true>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, ctr, big,
                                    (unsigned int *)(ctr + 6), big_cap);
                    }
                    unsigned long long hist[7];  // the histogram (label_count_kernel), [6]: the long lists
                    HIP_CHECK(hipMemcpyAsync(hist, ctr, 7 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
                    HIP_CHECK(hipStreamSynchronize(stream));
                    uint32_t nbig = (uint32_t)(hist[6] & 0xFFFFFFFFull);
                    if (nbig > big_cap && n) {
                        // more long lists than the first guess held (config #3's deep folder
                        // chains): the count pass again with room for all of them
                        big_cap = nbig;
                        big = dalloc<uint32_t>(big_cap);
                        tmp.push_back(big);
                        HIP_CHECK(hipMemsetAsync(ctr, 0, 8 * sizeof(unsigned long long), stream));
                        if (side == 0)
                            KLAUNCH(label_count_kernel<false>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, ctr, big,
                                    (unsigned int *)(ctr + 6), big_cap);
                        else
                            KLAUNCH(label_count_kernel<true>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, ctr, big,
                                    (unsigned int *)(ctr + 6), big_cap);
                        HIP_CHECK(hipMemcpyAsync(hist, ctr, 7 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
                        HIP_CHECK(hipStreamSynchronize(stream));
                        nbig = (uint32_t)(hist[6] & 0xFFFFFFFFull);
                        if (nbig > big_cap) throw Error(KETOGPU_EDEVICE, "plan label: long-list count changed between passes");
                    }
                    // the host's nodes: their lists (label_list), their counts into cnt
                    std::vector<uint32_t> hbig(nbig), hcnt(nbig);
                    std::vector<std::vector<uint32_t>> blist(nbig);
                    std::vector<uint64_t> bmask(nbig);
                    if (nbig) {
                        HIP_CHECK(hipMemcpy(hbig.data(), big, nbig * 4, hipMemcpyDeviceToHost));
                        parallel_chunks(nbig, 64, [&](int, uint64_t b, uint64_t e) {
                            for (uint64_t k = b; k < e; k++) {
                                label_list(s, *R, side == 1, hbig[k], blist[k], bmask[k]);
                                hcnt[k] = (uint32_t)blist[k].size();
                            }
                        });
                        uint32_t *dc = dalloc<uint32_t>(nbig);
                        tmp.push_back(dc);
                        HIP_CHECK(hipMemcpy(dc, hcnt.data(), nbig * 4, hipMemcpyHostToDevice));
                        KLAUNCH(label_big_io_kernel, dim3((nbig + 255) / 256), dim3(256), 0, stream, big, nbig, cnt, dc,
                                nullptr, nullptr);
                    }
                    uint64_t ne = hist[0], fit[4] = {hist[1], hist[2], hist[3], hist[4]};
                    for (uint32_t c : hcnt) {  // (as the host build counts them)
                        ne += c != 0;
                        for (int k = 0; k < 4; k++) fit[k] += c != 0 && c <= (8u << k) - kHeadFixed;
                    }
                    if (!H[side]) H[side] = pick_head(ne, fit);
                    if (side == 0) nonempty_s = ne;
                    const uint32_t h = H[side], cap = h - kHeadFixed;
                    // the overflow lists' starts: block totals, scanned on the host, then per node
                    const uint64_t per = (uint64_t)kLabelScanPer * kLabelScanBlock;
                    const uint32_t nb = (uint32_t)std::max<uint64_t>((n + per - 1) / per, 1);
                    unsigned long long *bs = dalloc<unsigned long long>(nb);
                    tmp.push_back(bs);
                    KLAUNCH(label_ov_sum_kernel, dim3(nb), dim3(kLabelScanBlock), 0, stream, cnt, n, cap, bs);
                    std::vector<unsigned long long> hb(nb);
                    HIP_CHECK(hipMemcpyAsync(hb.data(), bs, nb * 8, hipMemcpyDeviceToHost, stream));
                    HIP_CHECK(hipStreamSynchronize(stream));
                    unsigned long long acc = 0;
                    for (auto &x : hb) {
                        const unsigned long long t = x;
                        x = acc;
                        acc += t;
                    }
                    const uint64_t base16 = ((uint64_t)n * h + 15) / 16, words = (base16 + acc) * 16;
                    if (base16 + acc >= (1ull << 32)) throw Error(KETOGPU_EINVAL, "plan label: head arrays pass 2^36 words");
                    used += 4 * words;
                    if (used > budget)
                        throw Error(KETOGPU_ENOMEM, "plan label: " + std::to_string(used) + "+ bytes of heads, budget " +
                                                        std::to_string(budget));
                    HIP_CHECK(hipMemcpy(bs, hb.data(), nb * 8, hipMemcpyHostToDevice));
                    KLAUNCH(label_ov_off_kernel, dim3(nb), dim3(kLabelScanBlock), 0, stream, cnt, n, cap, bs, base16,
                            off16);
                    uint32_t *arr = dalloc<uint32_t>(words);
                    owned.push_back(arr);
                    A[side] = arr;
                    label_nwords[side] = words;
                    label_bytes += 4 * words;
                    HIP_CHECK(hipMemsetAsync(arr, 0xFF, words * 4, stream));
                    HIP_CHECK(hipMemsetAsync(ctr, 0, 8 * sizeof(unsigned long long), stream));
                    if (n) {
                        if (side == 0)
                            KLAUNCH(label_write_kernel<false>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, off16, arr,
                                    h, permille, ctr);
                        else
                            KLAUNCH(label_write_kernel<true>, dim3(grid), dim3(256), 0, stream, g, D, n, cnt, off16, arr,
                                    h, 0u, ctr);
                    }
                    if (nbig) {  // the host's nodes: overflow starts down, records up, one patch launch
                        uint32_t *doff = dalloc<uint32_t>(nbig);
                        tmp.push_back(doff);
                        KLAUNCH(label_big_io_kernel, dim3((nbig + 255) / 256), dim3(256), 0, stream, big, nbig, cnt,
                                nullptr, off16, doff);
                        std::vector<uint32_t> hoff(nbig);
                        HIP_CHECK(hipMemcpyAsync(hoff.data(), doff, nbig * 4, hipMemcpyDeviceToHost, stream));
                        HIP_CHECK(hipStreamSynchronize(stream));
                        std::vector<uint32_t> rec;
                        std::vector<uint64_t> roff(nbig);
                        for (uint32_t k = 0; k < nbig; k++) {
                            roff[k] = rec.size();
                            const uint32_t c = hcnt[k];
                            const bool inl = c <= cap;
                            const bool nl = side == 0 && c && label_nolabel(hbig[k], permille);
                            rec.push_back(hbig[k]);
                            rec.push_back(c);
                            const size_t hd = rec.size();
                            rec.resize(hd + h, 0xFFFFFFFFu);
                            rec[hd] = nl ? kNoLabel : c;
                            rec[hd + 1] = inl ? 0u : hoff[k];
                            rec[hd + 2] = (uint32_t)bmask[k];
                            rec[hd + 3] = (uint32_t)(bmask[k] >> 32);
                            std::copy(blist[k].begin(), blist[k].begin() + std::min<size_t>(c, cap),
                                      rec.begin() + (ptrdiff_t)(hd + kHeadFixed));
                            if (!inl) rec.insert(rec.end(), blist[k].begin(), blist[k].end());
                            nolabel += nl;
                            if (side == 0) s_entries += c;
                        }
                        uint32_t *drec = dalloc<uint32_t>(rec.size());
                        uint64_t *droff = dalloc<uint64_t>(nbig);
                        tmp.push_back(drec);
                        tmp.push_back(droff);
                        HIP_CHECK(hipMemcpy(drec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
                        HIP_CHECK(hipMemcpy(droff, roff.data(), nbig * 8, hipMemcpyHostToDevice));
                        KLAUNCH(label_patch_kernel, dim3(std::min<uint32_t>(nbig, 4096)), dim3(64), 0, stream, drec, droff,
                                nbig, arr, h);
                    }
                    unsigned long long tally[3];
                    HIP_CHECK(hipMemcpyAsync(tally, ctr, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
                    HIP_CHECK(hipStreamSynchronize(stream));
                    if (s.writable) {  // what label_update needs: every node's storage (counts, overflow starts)
                        std::vector<uint32_t> &cap_v = lab_cap[side], &ovf_v = lab_ovf[side];
                        cap_v.resize(n);
                        ovf_v.resize(n);
                        if (n) {
                            HIP_CHECK(hipMemcpy(cap_v.data(), cnt, (size_t)n * 4, hipMemcpyDeviceToHost));
                            HIP_CHECK(hipMemcpy(ovf_v.data(), off16, (size_t)n * 4, hipMemcpyDeviceToHost));
                        }
                        for (uint32_t x = 0; x < n; x++) cap_v[x] = cap_v[x] <= cap ? cap : (cap_v[x] + 15) / 16 * 16;
                    }
                    if (side == 0) {
                        s_entries += tally[0];
                        nolabel += tally[1];
                    }
                    label_overflow_share[side] = ne ? (double)(tally[2] + nbig) / (double)ne : 0.0;
                    if (cascade_log)
                        fprintf(stderr, "[label] %s heads: %u nodes, %u words each, %llu lists in overflow, %u long lists "
                                        "built on the host, %.2f GB\n",
                                side == 0 ? "S" : "P", n, h, (unsigned long long)tally[2] + (unsigned long long)nbig,
                                nbig, 4.0 * (double)words / 1e9);
                    free_tmp_side(tmp, {cnt, off16, big});
                }
                free_tmp();
                if (s.writable) lab_R = R;
            }
        } catch (const Error &e) {
            fprintf(stderr, "[ketogpu] plan label disabled: %s\n", e.what());
            free_tmp();
            release_label(A);
            drop_label();
            return;
        } catch (const std::bad_alloc &) {
            fprintf(stderr, "[ketogpu] plan label disabled: out of host memory\n");
            free_tmp();
            release_label(A);
            drop_label();
            return;
        }
        if (!rest_counts) {
            rest_counts = dalloc<unsigned int>(2 * kLabelSets * kRestShards * kRestStride);
            owned.push_back(rest_counts);
            HIP_CHECK(hipMemset(rest_counts, 0, 2 * kLabelSets * kRestShards * kRestStride * sizeof(unsigned int)));
        }
        lgraph = LabelGraph{A[1], A[0], s.Ni};
        if (s.writable) {
            if (!lab_R) {  // (the host build path: labels and storage from the snapshot again)
                lab_R = reach_labels_of(s);
                for (int side = 0; side < 2; side++) {
                    const uint64_t n = side == 0 ? label_s_nodes(s) : s.Nx;
                    std::vector<uint32_t> hd((size_t)n * H[side]);
                    if (n) HIP_CHECK(hipMemcpy(hd.data(), A[side], hd.size() * 4, hipMemcpyDeviceToHost));
                    lab_cap[side].resize(n);
                    lab_ovf[side].resize(n);
                    for (uint64_t x = 0; x < n; x++) {
                        const uint32_t c = hd[x * H[side]], o = hd[x * H[side] + 1];
                        lab_ovf[side][x] = o;
                        lab_cap[side][x] = o && c != kNoLabel ? (c + 15) / 16 * 16 : H[side] - kHeadFixed;
                    }
                }
            }
            lab_succ.resize(s.Ni);
            for (uint32_t v = 0; v < s.Ni; v++) lab_succ[v] = succ_hash(s, v);
            lab_pinv.assign(s.Nx, 0);
            lab_invalid = 0;
            lab_permille = permille;
        }
        label_hs = H[0];
        label_hp = H[1];
        label_coverage = nonempty_s ? 1.0 - (double)nolabel / (double)nonempty_s : 1.0;
        label_nolabel_heads = nolabel;
        label_knob = permille;
        if (getenv("KETOGPU_LABEL_HOST")) {
            uint64_t ne = 0;
            for (uint64_t x = 0; x < s.N; x++) ne += s.rev_off[x + 1] > s.rev_off[x];
            label_coverage = ne ? 1.0 - (double)nolabel / (double)ne : 1.0;
        }
        // the plan; neither plan core nor the hubs are built.  Without trials — unless (auto)
        // a quarter or more of one side's lists overflow their heads: the dense pass would
        // then answer many requests, so the first batches of >= kTrialMin requests also time
        // plan lite (the traversal over the records, no index) and the faster one is kept
        use_core = false;
        use_bidi = true;
        bidi_cfg = BidiCfg{9, 64, kLiteF, 7, 16, 1, 3};
        trials_left = 0;
        candidates.clear();
        if (plan_auto && use_lite && std::max(label_overflow_share[0], label_overflow_share[1]) >= 0.25) {
            candidates.push_back({true, 9, 64, kLiteF, 7, 0, true, 16, 1, 3});  // plan label
            candidates.push_back({true, 9, 64, kLiteF, 7, 0, true, 16, 1, 1});  // plan lite
            trials_left = kTrialRuns;
        }
        label_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (cascade_log)
            fprintf(stderr, "[label] %u landmarks, %llu label entries (%.1f ms); S heads %u words (%llu entries), P heads "
                            "%u words; %.2f GB; built in %.1f ms\n",
                    s.Ni, (unsigned long long)label_entries, label_pll_ms, label_hs, (unsigned long long)s_entries,
                    label_hp, (double)label_bytes / 1e9, label_build_ms);
    }
    // a build's temporaries freed early (the side's counts and offsets)
    static void free_tmp_side(std::vector<void *> &tmp, std::initializer_list<void *> ps) {
        for (void *p : ps) {
            auto it = std::find(tmp.begin(), tmp.end(), p);
            if (it != tmp.end()) {
                (void)hipFree(p);
                tmp.erase(it);
            }
        }
    }
    // a failed build's head arrays
    void release_label(uint32_t *(&A)[2]) {
        for (uint32_t *&p : A)
            if (p) {
                owned.erase(std::remove(owned.begin(), owned.end(), (void *)p), owned.end());
                (void)hipFree(p);
                p = nullptr;
            }
    }

    // Hub index.  Hubs are the interior nodes with the most interior successors; a search
    // (global path, unit2 kernels) marks a hub visited but does not expand it, and the pull
    // finds v in X(r) when v is in the closure of a hub the request reached (hub_mask,
    // precomputed once per engine).  On power-law nesting (BASELINE config #4) the closures
    // of popular groups cover most of the graph, while the search that stops at the hubs
    // stays small: with every interior node of >= kHubDeg interior successors a hub, the
    // non-hub branching factor drops below one.  KETOGPU_HUBS = number of hubs (0 = off);
    // default: on for graphs with >= 1024 interior nodes and an interior row of >= 64
    // entries, H = those nodes rounded up to 64, at most 65536 and at most 1/8 of free HBM
    // for hub_mask (Ni * H / 8 bytes).  Off with ambiguous keys: R4 flags are raised by the
    // rows a search reads, and a hub's closure is not read.
    static constexpr uint64_t kHubDeg = 8;
    std::vector<uint32_t> hub_nodes, hub_of_h;
    void choose_hubs(const Snapshot &s) {
        // writable snapshots: an in-place write would change hub closures (no hub index);
        // plan label answers without searches (KETOGPU_HUBS still forces the index)
        if (s.has_ambiguous || !s.Ni || s.writable) return;
        if (use_label && !getenv("KETOGPU_HUBS")) return;
        auto deg = [&](uint32_t v) { return s.fint_off[v + 1] - s.fint_off[v]; };
        uint64_t maxdeg = 0, heavy = 0;
        for (uint32_t v = 0; v < s.Ni; v++) {
            maxdeg = std::max<uint64_t>(maxdeg, deg(v));
            heavy += deg(v) >= kHubDeg;
        }
        uint64_t want = s.Ni >= 1024 && maxdeg >= 64 ? std::min<uint64_t>((heavy + 63) / 64 * 64, 65536) : 0;
        if (const char *e = getenv("KETOGPU_HUBS")) want = (uint64_t)std::max(0, atoi(e));
        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        want = std::min<uint64_t>(want, (uint64_t)free_b / 8 / ((uint64_t)s.Ni * 8) * 64);
        if (!want) return;
        std::vector<uint32_t> cand;
        for (uint32_t v = 0; v < s.Ni; v++)
            if (deg(v) >= 2) cand.push_back(v);
        const uint32_t H = (uint32_t)std::min<size_t>(want, cand.size());
        if (!H) return;
        std::partial_sort(cand.begin(), cand.begin() + H, cand.end(), [&](uint32_t a, uint32_t b) {
            return deg(a) != deg(b) ? deg(a) > deg(b) : a < b;
        });
        cand.resize(H);
        hub_of_h.assign(s.Nx, KETOGPU_NODE_NONE);
        for (uint32_t i = 0; i < H; i++) hub_of_h[cand[i]] = i;
        hub_nodes = std::move(cand);
        hub_words = (H + 63) / 64;
    }
    // the hub closures: one request per hub (root = target = the hub) on the global path
    // with the hub index still off; vis rows are copied into hub_mask per round
    void build_hubs(const Snapshot &s) {
        const uint32_t H = (uint32_t)hub_nodes.size();
        if (!H) return;
        auto t0 = std::chrono::steady_clock::now();
        uint32_t *d_r = dupload(hub_nodes);
        uint64_t *d_a = dalloc<uint64_t>(hub_words), *d_f = dalloc<uint64_t>(hub_words);
        hub_mask = dalloc<uint64_t>((size_t)s.Ni * hub_words);
        owned.push_back(hub_mask);
        HIP_CHECK(hipMemsetAsync(hub_mask, 0, (size_t)s.Ni * hub_words * 8, stream));
        HIP_CHECK(hipMemsetAsync(d_f, 0, hub_words * 8, stream));
        Batch b;
        b.roots = d_r;
        b.targets = d_r;
        b.n = H;
        b.allowed = d_a;
        b.flags = d_f;
        ketogpu_run_stats rs{};
        std::vector<std::pair<hipEvent_t, hipEvent_t>> pe, qe;
        ev_used = 0;
        run_global(b, rs, pe, qe, true);
        HIP_CHECK(hipStreamSynchronize(stream));
        for (void *p : {(void *)d_r, (void *)d_a, (void *)d_f}) (void)hipFree(p);
        st.hub_of = up_hub(hub_of_h);
        st.hub_mask = hub_mask;
        st.hub_reach = dalloc<uint64_t>((size_t)Wmax * 64 * hub_words);
        owned.push_back(st.hub_reach);
        st.hub_words = hub_words;
        g.hub_of = st.hub_of;
        g.hub_mask = hub_mask;
        g.hub_words = hub_words;
        n_hubs = H;
        hub_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (cascade_log)
            fprintf(stderr, "[hubs] %u hubs (interior rows >= %llu entries: smallest hub row %llu) built in %.1f ms\n",
                    H, (unsigned long long)kHubDeg,
                    (unsigned long long)(s.fint_off[hub_nodes.back() + 1] - s.fint_off[hub_nodes.back()]), hub_build_ms);
        std::vector<uint32_t>().swap(hub_of_h);
        // with hubs, the multi-word global path alone is a candidate of the auto plan (on
        // power-law graphs it beats the LDS stages, whose tables the big closures overflow)
        if (trials_left && use_units) candidates.push_back({false, 0, 0, 0, 0, 0, false});
    }
    const uint32_t *up_hub(const std::vector<uint32_t> &v) {
        uint32_t *p = dupload(v);
        owned.push_back(p);
        return p;
    }

    // spill lists hold unit ids (at most one per request); spill_units has two halves
    // used as the ping-pong lists of the cascade
    void ensure_spill(uint64_t n) {
        if (n <= spill_cap) return;
        // (a queued call on either stream may still read the lists: let them finish first)
        if (pipe_busy() || pipe_q[0]) HIP_CHECK(hipDeviceSynchronize());
        for (void *p : {(void *)spill_units, (void *)spill_roots, (void *)spill_targets, (void *)spill_allowed,
                        (void *)spill_flags})
            if (p) (void)hipFree(p);
        // (+ 2048: plan label's sharded rest list rounds every shard's region up to whole units)
        spill_cap = std::max<uint64_t>(n + 2048, 1024);
        spill_units = dalloc<uint32_t>(2 * spill_cap);  // two ping-pong lists
        if (full_rec) (void)hipFree(full_rec);
        full_rec = dalloc<uint4>(kLabelSets * 2 * spill_cap);  // two records per listed request, per set
        spill_roots = dalloc<uint32_t>(spill_cap);
        spill_targets = dalloc<uint32_t>(spill_cap);
        spill_allowed = dalloc<uint64_t>(spill_cap / 64 + 1);
        spill_flags = dalloc<uint64_t>(spill_cap / 64 + 1);
    }

    // sum the spread unit-statistics slots (rows, edges, reverse entries)
    unsigned long long *stat_out() { return st.stats + 8 + 8 * kStatSlots; }

    // sum the spread unit-statistics slots of both regions (rows, edges, reverse entries)
    void read_unit_stats(uint64_t out[3]) {
        KLAUNCH(stats_reduce_kernel, dim3(1), dim3(kBlock), 0, stream, st.stats + 8, 2, stat_out(), nullptr, 0,
                EmitReq{});
        HIP_CHECK(hipMemcpyAsync(h_ctr + 32, stat_out(), 6 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
        for (int k = 0; k < 3; k++) out[k] = h_ctr[32 + k] + h_ctr[35 + k];
    }

    uint32_t read_spill_count() {
        HIP_CHECK(hipMemcpyAsync(h_ctr + 12, spill_count, sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
        return (uint32_t)h_ctr[12];
    }

    // After a bidi first stage over the whole batch q (its spilled units in list[0],
    // counted in spill_count[0]; events a -> b around it): the spill stages of `cascade`
    // (persistent over the previous stage's spilled units, counts read on the device),
    // the statistics reduction and ONE host synchronization.  `before_sync` enqueues
    // more work (result copies) ahead of that synchronization.  Returns the number of
    // single requests left in spill_units[0..) for the global path.
    uint64_t bidi_tail(const Batch &q, ketogpu_run_stats &rs, std::vector<std::pair<hipEvent_t, hipEvent_t>> &unit_ev,
                       hipEvent_t a, hipEvent_t b, uint64_t bunits, const std::function<void()> &before_sync = {}) {
        uint32_t *list[2] = {spill_units, spill_units + spill_cap};
        hipEvent_t d = ev();
        // spill stages of no more requests per unit than the stage before (an 8-request
        // first stage skips the 16-request stage w)
        std::vector<SpillStage> stages;
        for (const SpillStage &sg : cascade)
            if (sg.u <= (stages.empty() ? bidi_cfg.u : stages.back().u)) stages.push_back(sg);
        int u_prev = bidi_cfg.u;
        std::vector<uint32_t> fans;
        for (const SpillStage &sg : stages) {
            fans.push_back((uint32_t)(u_prev / sg.u));
            u_prev = sg.u;
        }
        if (bidi_cfg.lite == 3) {  // plan label: the first stage lists single requests; one stage after it
            stages.assign(1, SpillStage{1, 'L'});
            fans.assign(1, 1u);
            u_prev = 1;
        }
        const int cur = (int)(stages.size() & 1);  // the list the last stage writes
        static const bool eager_env = getenv("KETOGPU_CASCADE_EAGER") != nullptr;
        // (plan label: the rest stage as lazily — label_full_kernel totals the rest list)
        const bool lazy = !eager_env && !cascade_log && stage_prev[0] == 0;
        const EmitReq E = emit_req;
        emit_req = EmitReq{};
        // a lean plan-label call (run_once: HBM-resident, events off, lazy rest stage): no
        // statistics launch, the dense pass writes the counters' mirror itself
        const bool fused = bidi_cfg.lite == 3 && lean_call;
        if (fused && (!lazy || E.out)) throw Error(KETOGPU_EDEVICE, "lean label call without a lazy rest stage");
        // plan label: the dense pass over the requests with an overflowing list, always (it
        // also totals the rest list for the lazy decision below: spill_count[0]); persistent,
        // its grid from the previous call's count
        if (bidi_cfg.lite == 3)
            label_dispatch([&](auto hs, auto hp) {
                const unsigned fg = (unsigned)std::min<uint64_t>(std::max<uint64_t>(full_prev / 16 + 64, 64), 16384);
                KLAUNCH((label_full_kernel<decltype(hs)::value, decltype(hp)::value>), dim3(fg), dim3(64), 0, stream,
                        lgraph, q.allowed, label_rest(q.n), label_full(q.n), &spill_count[0], &spill_count[7],
                        fused ? nullptr : st.stats + 4 * kStatSlots, fused ? d_hctr + 16 : nullptr);
            });
        if (fused && pipelined_req && !trials_left && label_rest_free(q)) {
            // a pipelined lean call (ketogpu_queries_run_async): no request of this batch can
            // be listed for the second stage (label_rest_free), so nothing after the dense pass
            // depends on the lists' totals: the call returns without a host wait.  The results
            // are complete when the stream is (ketogpu_queries_download, ketogpu_engine_wait);
            // the counters are left as a lean call without rest requests leaves them
            queued = true;
            unit_end = d;
            rs.rest_requests = 0;
            rs.full_requests = full_prev;  // (not read back: the last synchronized call's count)
            label_clean = true;
            label_calls++;
            rs.push_launches += 2;
            rs.unit_launches += 2;
            return 0;
        }
        auto launch_stages = [&](uint64_t prev0) {
            for (size_t k = 0, c = 0; k < stages.size(); k++, c ^= 1)
                launch_stage(stages[k], q, list[c], &spill_count[k], fans[k], list[c ^ 1], &spill_count[k + 1],
                             st.stats + 4 * kStatSlots, k == 0 ? prev0 : k < 8 ? stage_prev[k] : ~0ull);
        };
        // Lazy cascade: when the previous call's first stage spilled nothing (config #2: one
        // unit in 60k, most calls none), the spill stages are not launched up front — three
        // empty persistent launches cost ~14 us per call — but only after the synchronization
        // shows spills, followed by a second statistics pass, the result copies again and a
        // second synchronization.  KETOGPU_CASCADE_EAGER=1: always up front (A/B).
        if (!lazy) launch_stages(stage_prev[0]);
        // b == nullptr (host batches): no event between the call's kernels (each costs ~6 us of
        // GPU idle between the launches it separates); one event after the last launch
        if (b) HIP_CHECK(hipEventRecord(d, stream));
        const size_t ns = stages.size() + 1;
        // the spill counters sit 8 words after the reduced statistics (st.stats
        // layout, kStatsLen): the reduction mirrors both into h_ctr[16..21] and h_ctr + 24
        // (host-mapped: no copy launch between it and the sync)
        static_assert(kStatsLen == 8 + 8 * kStatSlots + 12, "statistics layout");
        // (ns <= 7: KETOGPU_CASCADE allows at most 6 stages; the block holds 8 counters)
        // a pending host-batch emit rides in the same launch (blocks >= 1)
        const unsigned eb = E.out ? (unsigned)std::min<uint64_t>(blocks_for(2 * E.words + 1), 255) : 0;
        if (!fused)
            KLAUNCH(stats_reduce_kernel, dim3(1 + eb), dim3(kBlock), 0, stream, st.stats + 8, 2, stat_out(), d_hctr + 16,
                    12, E);
        if (before_sync) before_sync();
        if (!b && !lean_call) HIP_CHECK(hipEventRecord(d, stream));
        wait_stream();
        const unsigned int *cnt = (const unsigned int *)(h_ctr + 24);
        size_t launched = lazy ? 1 : stages.size() + 1;
        if (lazy && cnt[0]) {  // spilled after all: the stages now, then statistics and results again
            d = ev();
            launch_stages((uint64_t)cnt[0] * fans[0]);
            KLAUNCH(stats_reduce_kernel, dim3(1 + eb), dim3(kBlock), 0, stream, st.stats + 8, 2, stat_out(),
                    d_hctr + 16, 12, E);
            if (before_sync) before_sync();
            if (!lean_call) HIP_CHECK(hipEventRecord(d, stream));
            wait_stream();
            launched = stages.size() + 2;
        }
        unit_end = d;
        if (b) {
            unit_ev.push_back({a, b});
            unit_ev.push_back({b, d});
        } else if (!lean_call) {
            unit_ev.push_back({a, d});
        }
        const uint64_t *t = (const uint64_t *)h_ctr + 16;
        rs.main_bytes = 16 * t[0] + 16 * t[1] + 4 * t[2] + 8 * q.n + 8 * ((q.n + 63) / 64);
        if (cascade_log) {
            fprintf(stderr, "[cascade] units %llu, spills per stage:", (unsigned long long)bunits);
            for (size_t k = 0; k < ns; k++) fprintf(stderr, " %u", cnt[k]);
            fprintf(stderr, "\n");
        }
        for (size_t k = 0; k < ns; k++) rs.spilled_units += cnt[k];
        if (bidi_cfg.lite == 3) {
            rs.rest_requests = cnt[0];
            rs.full_requests = cnt[7];
            full_prev = cnt[7];
            // a lean call without rest requests touched no statistics slot and no spill
            // counter past [0] and [7] (both written, not added to): the next call needs no clear
            label_clean = fused && cnt[0] == 0;
        }
        for (size_t k = 0; k < stages.size() && k < 8; k++) stage_prev[k] = (uint64_t)cnt[k] * fans[k];
        rs.push_launches += launched;
        rs.unit_launches += launched;
        const uint64_t left = cnt[ns - 1];
        if (u_prev != 1) throw Error(KETOGPU_EINVAL, "bidi cascade must end with a single-request stage");
        if (bidi_cfg.lite == 3) label_calls++;  // the next call uses the next counter set
        if (left && cur != 0)  // single requests for the global path, read from list[0]
            HIP_CHECK(hipMemcpyAsync(list[0], list[cur], left * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
        return left;
    }

    // The LDS cascade: 16-request units, then 4-request and 1-request units for what
    // spilled.  Returns the number of single requests left in spill_units[0..) for the
    // global path.
    // The end of a run.  KETOGPU_WAIT=spin: poll an event recorded after the last launch
    // (the host thread busy-waits, no wake-up latency); default: hipStreamSynchronize.
    hipEvent_t wait_ev = nullptr;
    void wait_stream() {
        static const bool spin = [] {
            const char *w = getenv("KETOGPU_WAIT");
            return w && !strcmp(w, "spin");
        }();
        if (!spin) {
            HIP_CHECK(hipStreamSynchronize(stream));
            return;
        }
        if (!wait_ev) HIP_CHECK(hipEventCreateWithFlags(&wait_ev, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(wait_ev, stream));
        for (;;) {
            const hipError_t e = hipEventQuery(wait_ev);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) HIP_CHECK(e);
            __builtin_ia32_pause();
        }
    }

    uint64_t run_units(const Batch &q, ketogpu_run_stats &rs, std::vector<std::pair<hipEvent_t, hipEvent_t>> &unit_ev,
                       const HostSrc *src = nullptr, const std::function<void()> &before_sync = {}) {
        ensure_spill(q.n);
        uint32_t *list[2] = {spill_units, spill_units + spill_cap};
        if (wave_u) {
            // pass 1: one wave per unit of wave_u requests; pass 2: spilled units as
            // single requests with a workgroup-wide table
            uint64_t units = (q.n + wave_u - 1) / wave_u;
            unsigned grid = (unsigned)((units + 3) / 4);
            HIP_CHECK(hipMemsetAsync(spill_count, 0, sizeof(unsigned int), stream));
            hipEvent_t a = ev(), b = ev();
            HIP_CHECK(hipEventRecord(a, stream));
            if (wave_u == 4)
                KLAUNCH((wave_unit_kernel<4, 9>), dim3(grid), dim3(kBlock), 0, stream, g, has_kids, q.roots,
                                   q.targets, q.n, q.allowed, q.flags, list[0], spill_count, st.stats);
            else if (wave_u == 8)
                KLAUNCH((wave_unit_kernel<8, 10>), dim3(grid), dim3(kBlock), 0, stream, g, has_kids,
                                   q.roots, q.targets, q.n, q.allowed, q.flags, list[0], spill_count, st.stats);
            else
                KLAUNCH((wave_unit_kernel<16, 11>), dim3(grid), dim3(kBlock), 0, stream, g, has_kids,
                                   q.roots, q.targets, q.n, q.allowed, q.flags, list[0], spill_count, st.stats);
            HIP_CHECK(hipEventRecord(b, stream));
            unit_ev.push_back({a, b});
            uint64_t left = read_spill_count();
            rs.spilled_units += left;
            rs.push_launches++;
            if (!left) return 0;
            HIP_CHECK(hipMemsetAsync(spill_count, 0, sizeof(unsigned int), stream));
            a = ev();
            b = ev();
            HIP_CHECK(hipEventRecord(a, stream));
            KLAUNCH(unit_kernel<1>, dim3((unsigned)(left * wave_u)), dim3(kBlock), 0, stream, g, has_kids,
                               q.roots, q.targets, q.n, q.allowed, q.flags, list[0], (uint32_t)wave_u, list[1],
                               spill_count, st.stats, nullptr);
            HIP_CHECK(hipEventRecord(b, stream));
            unit_ev.push_back({a, b});
            left = read_spill_count();
            rs.spilled_units += left;
            rs.push_launches++;
            if (left)
                HIP_CHECK(hipMemcpyAsync(list[0], list[1], left * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
            return left;
        }
        uint64_t units = (q.n + 15) / 16;
        uint64_t left = 0;
        if (use_v2 || (use_lite && use_bidi)) {
            // Forward-only plan "v2": the host-driven unit2 cascade unit2<16> -> unit2<4> ->
            // unit2<1> -> global path.
            if (use_bidi) {
                // bidi (configured shape) over every unit, then the spill stages of
                // `cascade` (persistent over the previous stage's spilled units, counts read
                // on the device), then the global path for single requests that exceed the
                // last table; one host synchronization for counts and statistics
                // host batches (src): the run's begin event was recorded ahead of its clear
                // launch (light_begin) and no event separates the call's kernels
                const bool direct = src && src->mapped && pipe_direct &&
                                    (bidi_cfg == BidiCfg{9, 64, KETO_F1, 7, 16, 1} || bidi_cfg.lite);
                // (the chunk pipeline's other streams wait for an event after the clear)
                const bool light = light_begin && (direct || !src);
                hipEvent_t a = light ? light_begin : ev(), b = light ? nullptr : ev();
                if (!light) HIP_CHECK(hipEventRecord(a, stream));
                const uint64_t bunits = (q.n + bidi_cfg.u - 1) / bidi_cfg.u;
                if (!src) {
                    launch_bidi(bidi_cfg, (unsigned)bunits, lds_pad, q, nullptr, nullptr, list[0], &spill_count[0],
                                lean_call ? nullptr : st.stats, stamps);  // (lean: no statistics atomics)
                } else if (direct) {
                    // pinned requests: one launch whose units read their requests in place.
                    // (Tried: only a share f of the units reading in place while load_kernel
                    // copied the rest into HBM for a second launch on stream2 — f = 0.25 /
                    // 0.35 / 0.5: 1.85 / 1.83 / 1.90 vs 2.09 x 10^9 checks/s,
                    // profiles/r02/ab_split.)
#define KETO_HOST_K(K)                                                                                     \
    do {                                                                                                   \
        if (bidi_cfg.lite == 3)                                                                            \
            launch_label_host(q, src, bunits);                                                             \
        else if (bidi_cfg.lite == 2 && core_shape == 1)                                                    \
            KLAUNCH((lite_host_kernel<K, CoreShapeS, true>), dim3((unsigned)((bunits + K - 1) / K)), dim3(64), \
                    0, stream, gcore(), core_rec[0], core_rec[1], src->roots, src->targets, io->d_roots,   \
                    io->d_targets, q.n, q.allowed, list[0], &spill_count[0], st.stats, d_bad);              \
        else if (bidi_cfg.lite == 2 && core_shape == 2)                                                    \
            KLAUNCH((lite_host_kernel<K, CoreShapeM, true>), dim3((unsigned)((bunits + K - 1) / K)), dim3(64), \
                    0, stream, gcore(), core_rec[0], core_rec[1], src->roots, src->targets, io->d_roots,   \
                    io->d_targets, q.n, q.allowed, list[0], &spill_count[0], st.stats, d_bad);              \
        else if (bidi_cfg.lite == 2)                                                                       \
            KLAUNCH((lite_host_kernel<K, LiteShape, true>), dim3((unsigned)((bunits + K - 1) / K)), dim3(64), \
                    0, stream, gcore(), core_rec[0], core_rec[1], src->roots, src->targets, io->d_roots,   \
                    io->d_targets, q.n, q.allowed, list[0], &spill_count[0], st.stats, d_bad);              \
        else if (bidi_cfg.lite && bidi_cfg.u == 32)                                                        \
            KLAUNCH((lite_host_kernel<K, LiteShape32>), dim3((unsigned)((bunits + K - 1) / K)), dim3(64), 0, \
                    stream, g, frec, brec, src->roots, src->targets, io->d_roots, io->d_targets, q.n,      \
                    q.allowed, list[0], &spill_count[0], st.stats, d_bad);                                 \
        else if (bidi_cfg.lite)                                                                            \
            KLAUNCH((lite_host_kernel<K, LiteShape>), dim3((unsigned)((bunits + K - 1) / K)), dim3(64), 0,   \
                    stream, g, frec, brec, src->roots, src->targets, io->d_roots, io->d_targets, q.n,      \
                    q.allowed, list[0], &spill_count[0], st.stats, d_bad);                                 \
        else                                                                                               \
            KLAUNCH(bidi_host_kernel<K>, dim3((unsigned)((bunits + K - 1) / K)), dim3(64), 0, stream, g,   \
                    frec, brec, src->roots, src->targets, io->d_roots, io->d_targets, q.n, q.allowed,      \
                    list[0], &spill_count[0], st.stats, d_bad);                                            \
    } while (0)
                    const int hk = host_units ? host_units : bidi_cfg.lite == 3 ? 4 : 2;
                    if (hk == 4)
                        KETO_HOST_K(4);
                    else if (hk == 2)
                        KETO_HOST_K(2);
                    else
                        KETO_HOST_K(1);
#undef KETO_HOST_K
                } else {
                    // Host-to-host batch (check_host): the requests arrive in chunks on the
                    // copy stream; each chunk is validated and its units launched as soon as
                    // it lands, alternating two streams so one chunk's tail overlaps the next
                    // chunk's start.  All chunks append spilled units to the one list, so the
                    // spill stages below run once for the whole batch.
                    HIP_CHECK(hipStreamWaitEvent(stream2, a, 0));  // after the clear
                    HIP_CHECK(hipStreamWaitEvent(copy_stream, a, 0));  // d_bad reset by the clear
                    const uint64_t U = (uint64_t)bidi_cfg.u;
                    // a short first chunk starts the traversal early; the rest in full chunks
                    uint64_t chunk = std::max<uint64_t>(64, pipe_chunk / 4 / 64 * 64);
                    for (uint64_t c0 = 0, k = 0; c0 < q.n; c0 += chunk, k++, chunk = pipe_chunk) {
                        const uint64_t m = std::min<uint64_t>(chunk, q.n - c0);
                        hipStream_t cs = (k & 1) ? stream2 : stream;
                        // the first chunk loads on the stream that traverses it (no cross-stream
                        // event ahead of the first launch: ~18 us idle); the others on the
                        // copy stream, overlapping the traversal of the chunks before them
                        hipStream_t ls = k ? copy_stream : cs;
                        if (src->mapped) {
                            KLAUNCH(load_kernel, dim3((unsigned)std::min<uint64_t>(blocks_for(m), 256)), dim3(kBlock), 0,
                                    ls, src->roots, src->targets, c0, m, io->d_roots, io->d_targets, g.Nx, g.N, d_bad);
                        } else {
                            HIP_CHECK(hipMemcpyAsync(io->d_roots + c0, src->roots + c0, m * 4, hipMemcpyDefault, ls));
                            HIP_CHECK(hipMemcpyAsync(io->d_targets + c0, src->targets + c0, m * 4, hipMemcpyDefault, ls));
                        }
                        if (k) {
                            hipEvent_t h = ev();
                            HIP_CHECK(hipEventRecord(h, copy_stream));
                            HIP_CHECK(hipStreamWaitEvent(cs, h, 0));
                        }
                        if (!src->mapped)
                            KLAUNCH(validate_kernel, dim3(blocks_for(m)), dim3(kBlock), 0, cs, io->d_roots + c0,
                                    io->d_targets + c0, m, g.Nx, g.N, c0, d_bad);
                        launch_bidi(bidi_cfg, (unsigned)((m + U - 1) / U), lds_pad, q, nullptr, nullptr, list[0],
                                    &spill_count[0], st.stats, nullptr, c0 / U, cs, true);
                    }
                    hipEvent_t j = ev();
                    HIP_CHECK(hipEventRecord(j, stream2));
                    HIP_CHECK(hipStreamWaitEvent(stream, j, 0));
                }
                if (b) HIP_CHECK(hipEventRecord(b, stream));
                return bidi_tail(q, rs, unit_ev, a, b, bunits, before_sync);
            }
            // Forward-only plan "v2": unit2<16> over every unit, then the persistent
            // unit2<4> and unit2<1> stages over the spilled units (counts read on the
            // device: no host synchronization between the stages; grids sized by the
            // previous call's counts, as the bidi cascade), one synchronization for the count
            // the global path needs.  list[0] <- 16 -> list[1] <- 4 -> list[0] <- 1.
            if (!units) return 0;
            unsigned int *c16 = spill_count + 2, *c4 = spill_count + 3, *c1 = spill_count + 4;
            HIP_CHECK(hipMemsetAsync(c16, 0, 3 * sizeof(unsigned int), stream));
            hipEvent_t a = ev(), b = ev();
            HIP_CHECK(hipEventRecord(a, stream));
            KLAUNCH(unit2_kernel<16>, dim3((unsigned)units), dim3(kBlock), lds_pad, stream, g, frec, q.roots, q.targets,
                    q.n, q.allowed, q.flags, nullptr, 1u, list[0], c16, st.stats, stamps);
            HIP_CHECK(hipEventRecord(b, stream));
            unit_ev.push_back({a, b});
            hipEvent_t c = ev();
            // KETOGPU_U2_SYNC=1 (A/B knob): the stages as one-unit-per-workgroup launches sized
            // by a host read of the previous stage's count (round 2's cascade)
            static const bool sync_stages = getenv("KETOGPU_U2_SYNC") != nullptr;
            if (sync_stages) {
                auto count = [&](unsigned int *cp) {
                    HIP_CHECK(hipMemcpyAsync(h_ctr + 12, cp, sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
                    HIP_CHECK(hipStreamSynchronize(stream));
                    return (uint64_t)*(const unsigned int *)(h_ctr + 12);
                };
                if (const uint64_t k = count(c16))
                    KLAUNCH(unit2_kernel<4>, dim3((unsigned)(k * 4)), dim3(kBlock), 0, stream, g, frec, q.roots,
                            q.targets, q.n, q.allowed, q.flags, list[0], 4u, list[1], c4, st.stats, nullptr);
                if (const uint64_t k = count(c4))
                    KLAUNCH(unit2_kernel<1>, dim3((unsigned)(k * 4)), dim3(kBlock), 0, stream, g, frec, q.roots,
                            q.targets, q.n, q.allowed, q.flags, list[1], 4u, list[0], c1, st.stats, nullptr);
            } else {
                // persistent grids: as many workgroups as fit the CUs at once (LDS-bound)
                constexpr unsigned per4 = (unsigned)(160 * 1024 / sizeof(Unit2Shared<4>));
                constexpr unsigned per1 = (unsigned)(160 * 1024 / sizeof(Unit2Shared<1>));
                static_assert(per4 >= 1 && per1 >= 1, "a unit2 stage's LDS exceeds a CU");
                KLAUNCH(unit2_cascade_kernel<4>, dim3(stage_grid(u2_prev[0], 256 * per4)), dim3(kBlock), 0, stream, g,
                        frec, q.roots, q.targets, q.n, q.allowed, q.flags, list[0], c16, 4u, list[1], c4, st.stats);
                KLAUNCH(unit2_cascade_kernel<1>, dim3(stage_grid(u2_prev[1], 256 * per1)), dim3(kBlock), 0, stream, g,
                        frec, q.roots, q.targets, q.n, q.allowed, q.flags, list[1], c4, 4u, list[0], c1, st.stats);
            }
            HIP_CHECK(hipEventRecord(c, stream));
            unit_ev.push_back({b, c});
            // the counts and the cascade's statistics (rows, edges, reverse entries: the first
            // stage dominates them) in one synchronization
            HIP_CHECK(hipMemcpyAsync(h_ctr + 12, c16, 3 * sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
            KLAUNCH(stats_reduce_kernel, dim3(1), dim3(kBlock), 0, stream, st.stats + 8, 2, stat_out(), nullptr, 0,
                    EmitReq{});
            HIP_CHECK(hipMemcpyAsync(h_ctr + 32, stat_out(), 6 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
            HIP_CHECK(hipStreamSynchronize(stream));
            const unsigned int *hc = (const unsigned int *)(h_ctr + 12);
            u2_prev[0] = (uint64_t)hc[0] * 4;
            u2_prev[1] = (uint64_t)hc[1] * 4;
            left = hc[2];
            rs.spilled_units += hc[0] + hc[1] + hc[2];
            rs.push_launches += 3;
            rs.unit_launches += 3;
            uint64_t t3[3];
            for (int k = 0; k < 3; k++) t3[k] = h_ctr[32 + k] + h_ctr[35 + k];
            rs.main_bytes = 16 * t3[0] + 16 * t3[1] + 4 * t3[2] + 8 * q.n + 8 * ((q.n + 63) / 64);
            return left;
        }
        for (int pass = 0; pass < 3; pass++) {
            uint64_t grid = pass == 0 ? units : left * 4;
            if (!grid) return 0;
            uint32_t *in = pass == 0 ? nullptr : list[(pass - 1) & 1], *out = list[pass & 1];
            HIP_CHECK(hipMemsetAsync(spill_count, 0, sizeof(unsigned int), stream));
            hipEvent_t a = ev(), b = ev();
            HIP_CHECK(hipEventRecord(a, stream));
            if (pass == 0)
                KLAUNCH(unit_kernel<16>, dim3((unsigned)grid), dim3(kBlock), 0, stream, g, has_kids, q.roots,
                                   q.targets, q.n, q.allowed, q.flags, nullptr, 1u, out, spill_count, st.stats, stamps);
            else if (pass == 1)
                KLAUNCH(unit_kernel<4>, dim3((unsigned)grid), dim3(kBlock), 0, stream, g, has_kids, q.roots,
                                   q.targets, q.n, q.allowed, q.flags, in, 4u, out, spill_count, st.stats, nullptr);
            else
                KLAUNCH(unit_kernel<1>, dim3((unsigned)grid), dim3(kBlock), 0, stream, g, has_kids, q.roots,
                                   q.targets, q.n, q.allowed, q.flags, in, 4u, out, spill_count, st.stats, nullptr);
            HIP_CHECK(hipEventRecord(b, stream));
            unit_ev.push_back({a, b});
            left = read_spill_count();
            rs.spilled_units += left;
            rs.push_launches++;
            rs.unit_launches++;
        }
        // the last pass wrote single requests into list[0]
        return left;
    }

    // read ctr[0..2] and overflow into h_ctr[0..3]
    void read_counters() {
        HIP_CHECK(hipMemcpyAsync(h_ctr, st.ctr, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipMemcpyAsync(h_ctr + 3, st.overflow, sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
    }

    // Global multi-word engine, one round over requests [c0, c0 + n) of batch q (c0 a
    // multiple of 64).  Returns false on list overflow (state is then dense-reset and
    // the caller splits the round).
    // hub_w0 != NONE: hub index build — the requests are hubs 64*hub_w0 ..., their
    // closures go to hub_mask instead of a pull
    bool round(const Batch &q, uint64_t c0, uint64_t n, ketogpu_run_stats &rs,
               std::vector<std::pair<hipEvent_t, hipEvent_t>> &push_ev,
               std::vector<std::pair<hipEvent_t, hipEvent_t>> &pull_ev, uint32_t hub_w0 = KETOGPU_NODE_NONE) {
        const uint64_t W = (n + 63) / 64;
        const uint64_t wg0 = c0 / 64;
        if (st.hub_reach) HIP_CHECK(hipMemsetAsync(st.hub_reach, 0, W * 64 * st.hub_words * 8, stream));
        HIP_CHECK(hipMemsetAsync(st.ctr, 0, 3 * sizeof(uint64_t), stream));
        HIP_CHECK(hipMemsetAsync(st.overflow, 0, sizeof(unsigned int), stream));
        *(uint64_t *)&h_ctr[3] = 0;
        KLAUNCH(seed_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.roots, q.targets, c0, n,
                           q.flags);
        read_counters();
        uint64_t cnt = h_ctr[0] >> kCntShift, edges = h_ctr[0] & kPreMask;
        std::vector<uint64_t> level_begin{0};
        uint64_t lb = 0;
        int cur = 0;  // ctr index of the current level
        if (q.has_dyn) {
            KLAUNCH(seed_dynamic_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.roots,
                               q.targets, c0, n, q.dyn_int_off, q.dyn_int, q.dyn_amb, q.flags, lb + cnt, &st.ctr[1]);
        }
        bool overflow = (uint32_t)h_ctr[3] != 0;
        for (uint64_t level = 0; !overflow; level++) {
            if (level > 0 && cnt)
                KLAUNCH(gather_kernel, dim3(blocks_for(cnt)), dim3(kBlock), 0, stream, g, st, lb, lb + cnt);
            bool dyn_pending = level == 0 && q.has_dyn;
            if (!cnt && !dyn_pending) break;
            int nxt = cur ^ 1;
            if (level > 0) HIP_CHECK(hipMemsetAsync(&st.ctr[nxt], 0, sizeof(uint64_t), stream));
            if (edges) {
                uint64_t tiles = (edges + kTile - 1) / kTile;
                unsigned grid = (unsigned)std::min<uint64_t>(tiles, 256ull * 16);
                hipEvent_t a = ev(), b = ev();
                HIP_CHECK(hipEventRecord(a, stream));
                KLAUNCH(expand_kernel, dim3(grid), dim3(kBlock), 0, stream, g, st, lb, cnt, edges, lb + cnt,
                                   &st.ctr[nxt], q.flags, wg0);
                HIP_CHECK(hipEventRecord(b, stream));
                push_ev.push_back({a, b});
                rs.push_launches++;
            }
            rs.levels++;
            rs.frontier_entries += cnt;
            rs.interior_edges += edges;
            read_counters();
            overflow = (uint32_t)h_ctr[3] != 0;
            uint64_t ncnt = h_ctr[nxt] >> kCntShift, nedges = h_ctr[nxt] & kPreMask;
            // algorithmic bytes of this push: 16 per row opened, 4 per edge, 8 per mask
            // read (entry mask + visited word per edge) and per mask write (new entries)
            rs.bytes_push += 16 * cnt + 4 * edges + 8 * (cnt + edges) + 8 * ncnt;
            lb += cnt;
            level_begin.push_back(lb);
            cnt = ncnt;
            edges = nedges;
            cur = nxt;
        }
        if (overflow) {
            size_t state = (size_t)Wmax * std::max<uint32_t>(g.Ni, 1);
            HIP_CHECK(hipMemsetAsync(st.vis, 0, state * 8, stream));
            HIP_CHECK(hipMemsetAsync(st.nxt, 0, state * 8, stream));
            HIP_CHECK(hipMemsetAsync(q.flags + wg0, 0, W * 8, stream));
            HIP_CHECK(hipStreamSynchronize(stream));
            return false;
        }
        if (hub_w0 != KETOGPU_NODE_NONE) {
            KLAUNCH(hub_mask_kernel, dim3(std::min<uint64_t>(blocks_for(W * g.Ni), 4096)), dim3(kBlock), 0, stream,
                    st.vis, g.Ni, W, hub_w0, hub_words, hub_mask);
        } else {
            hipEvent_t a = ev(), b = ev();
            HIP_CHECK(hipEventRecord(a, stream));
            KLAUNCH(pull_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.roots, q.targets, c0, n,
                    q.dyn_full_off, q.dyn_full, q.allowed);
            HIP_CHECK(hipEventRecord(b, stream));
            pull_ev.push_back({a, b});
        }
        // reset every visited entry recorded in this round (levels >= 1 and touch list)
        uint64_t first = level_begin.size() > 1 ? level_begin[1] : lb;
        if (lb > first)
            KLAUNCH(reset_kernel, dim3(blocks_for(lb - first)), dim3(kBlock), 0, stream, st.vis, g.Ni,
                               st.fe_key + first, lb - first);
        uint64_t ntouch = h_ctr[2];
        if (ntouch)
            KLAUNCH(reset_kernel, dim3(blocks_for(ntouch)), dim3(kBlock), 0, stream, st.vis, g.Ni, st.touch,
                               ntouch);
        rs.touched += (lb - first) + ntouch;
        rs.rounds++;
        return true;
    }

    void run_global(const Batch &q, ketogpu_run_stats &rs, std::vector<std::pair<hipEvent_t, hipEvent_t>> &push_ev,
                    std::vector<std::pair<hipEvent_t, hipEvent_t>> &pull_ev, bool hub_build = false) {
        uint64_t words = (q.n + 63) / 64;
        uint64_t W = Wmax;
        for (uint64_t w0 = 0; w0 < words;) {
            uint64_t wn = std::min<uint64_t>(W, words - w0);
            uint64_t c0 = w0 * 64, n = std::min<uint64_t>(q.n - c0, wn * 64);
            if (!round(q, c0, n, rs, push_ev, pull_ev, hub_build ? (uint32_t)w0 : KETOGPU_NODE_NONE)) {
                rs.overflow_retries++;
                if (wn == 1) throw Error(KETOGPU_ENOMEM, "frontier list overflow for a single 64-request word");
                W = std::max<uint64_t>(1, wn / 2);
                continue;
            }
            w0 += wn;
        }
    }

    void run(ketogpu_queries &qq) {
        HIP_CHECK(hipSetDevice(device));
        if (trials_left && qq.n >= kTrialMin) {
            const size_t nc = candidates.size();
            auto select = [&](const Candidate &c) {
                use_units = c.units;
                if (!c.units) return;
                use_bidi = c.bidi;
                bidi_cfg = BidiCfg{c.hlog, c.bt, c.f, c.lf, c.u, c.wpe, c.lite};
            };
            for (size_t k = 0; k < nc; k++) {
                Candidate &c = candidates[(k + (size_t)trials_left) % nc];  // rotate the order per trial
                select(c);
                run_once(qq);
                c.ms += last.ms_total;
            }
            if (--trials_left == 0) {
                size_t best = 0;
                for (size_t k = 1; k < nc; k++)
                    if (candidates[k].ms < candidates[best].ms) best = k;
                select(candidates[best]);
            }
            return;
        }
        run_once(qq);
    }

    // src: the requests are still on the host (check_host's pipelined first stage copies
    // them in); before_sync: copies enqueued ahead of the first-stage synchronization
    void run_once(ketogpu_queries &qq, const HostSrc *src = nullptr, const std::function<void()> &before_sync = {}) {
        Batch q = qq.batch();
        ketogpu_run_stats rs{};
        rs.checks = q.n;
        rs.plan = !use_units ? 0
                  : wave_u    ? 3
                  : use_bidi  ? (bidi_cfg.lite == 3 ? 7 : bidi_cfg.lite == 2 ? 6 : bidi_cfg.lite ? 5 : 1)
                  : use_v2    ? 2
                              : 4;
        rs.plan_lists = use_units && !wave_u && use_bidi ? (uint32_t)bidi_cfg.f : 0;
        rs.plan_unit = use_units && !wave_u && use_bidi ? (uint32_t)bidi_cfg.u : 0;
        rs.hubs = n_hubs;
        rs.hub_words = hub_words;
        rs.hub_build_ms = hub_build_ms;
        rs.closure_cap_f = use_core ? closure_cap[0] : 0;
        rs.closure_cap_b = use_core ? closure_cap[1] : 0;
        rs.closure_nodes_f = closure_nodes[0];
        rs.closure_nodes_b = closure_nodes[1];
        rs.closure_entries_f = closure_entries[0];
        rs.closure_entries_b = closure_entries[1];
        rs.core_build_ms = core_build_ms;
        rs.label_on = use_label ? 1 : 0;
        rs.label_s_head = use_label ? label_hs : 0;
        rs.label_p_head = use_label ? label_hp : 0;
        rs.label_coverage = label_coverage;
        rs.label_build_ms = label_build_ms;
        rs.label_pll_ms = label_pll_ms;
        rs.label_bytes = label_bytes;
        rs.label_entries = label_entries;
        rs.label_rewritten = lab_rewritten;
        rs.label_marked = lab_invalid;
        rs.label_relabels = lab_relabels;
        ev_used = 0;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> push_ev, pull_ev;
        hipEvent_t t_begin = ev(), t_end = ev();
        uint64_t words = (q.n + 63) / 64;
        // host batches: the run's begin event ahead of the clear launch (no event between
        // the call's kernels, KETOGPU_EVENTS=all restores them)
        // a lean call (HBM-resident plan label, events off: see lean_call) records no timing
        // event at all; its ms_total is the host's clock around the call
        const bool label_resident = !src && use_units && !wave_u && use_bidi && bidi_cfg.lite == 3 && q.n;
        static const bool eager_env = getenv("KETOGPU_CASCADE_EAGER") != nullptr;
        lean_call = label_resident && fuse_reduce && light_events && !eager_env && !cascade_log && stage_prev[0] == 0;
        const auto h0 = std::chrono::steady_clock::now();
        light_begin = nullptr;
        if (light_events && (src || (use_units && !wave_u && use_bidi && q.n && bidi_cfg.lite == 3))) {
            if (!lean_call) HIP_CHECK(hipEventRecord(t_begin, stream));
            light_begin = t_begin;  // (lean: never recorded, never read)
        }
        // one launch zeroes results, flags, statistics and spill counters — unless this is
        // a lean call after one that left them zero (label_kernel writes every result word
        // itself, a lean call adds no statistics)
        const bool skip_clear = lean_call && label_clean && qq.flags_zero && !clear_bad;
        label_clean = false;
        qq.flags_zero = false;
        if (!skip_clear)
            KLAUNCH(clear_kernel, dim3(64), dim3(kBlock), 0, stream, q.allowed, std::max<uint64_t>(words, 1),
                    q.flags, std::max<uint64_t>(words, 1), st.stats, (uint64_t)kStatsLen, clear_bad);
        clear_bad = nullptr;
        // A timing event costs ~5.6 us of GPU idle between the kernels it separates
        // (kernel trace of config #2): with the bidi first stage the run starts at that
        // stage's own start event, recorded right after this point.
        const bool bidi_first = use_units && !wave_u && (use_v2 || use_lite) && use_bidi && q.n;
        if (!bidi_first && !light_begin) HIP_CHECK(hipEventRecord(t_begin, stream));
        std::vector<std::pair<hipEvent_t, hipEvent_t>> unit_ev;
        if (use_units && q.n) {
            uint64_t ns = run_units(q, rs, unit_ev, src, before_sync);
            if (bidi_first && !lean_call) {
                if (!unit_ev.empty())
                    t_begin = unit_ev.front().first;
                else
                    HIP_CHECK(hipEventRecord(t_begin, stream));
            }
            rs.spilled_requests = ns;
            if (ns) {  // single requests whose closure exceeds an LDS table: global path
                KLAUNCH(spill_gather_kernel, dim3(blocks_for(ns)), dim3(kBlock), 0, stream, spill_units, ns,
                                   q.roots, q.targets, q.n, spill_roots, spill_targets);
                Batch sb = q;
                sb.roots = spill_roots;
                sb.targets = spill_targets;
                sb.n = ns;
                sb.allowed = spill_allowed;
                sb.flags = spill_flags;
                HIP_CHECK(hipMemsetAsync(spill_flags, 0, (ns / 64 + 1) * 8, stream));
                HIP_CHECK(hipMemsetAsync(spill_allowed, 0, (ns / 64 + 1) * 8, stream));
                run_global(sb, rs, push_ev, pull_ev);
                KLAUNCH(spill_scatter_kernel, dim3(blocks_for(ns)), dim3(kBlock), 0, stream, spill_units, ns,
                                   spill_allowed, spill_flags, q.allowed, q.flags);
            }
        } else {
            run_global(q, rs, push_ev, pull_ev);
        }
        uint64_t t3[3];
        uint64_t examined = 0;
        if (use_units && !wave_u && use_bidi && q.n && !rs.spilled_requests) {
            // bidi cascade without global-path requests: run_units already synchronized,
            // reduced and read the unit statistics (one host synchronization per run)
            t_end = unit_end;
            const uint64_t *t = (const uint64_t *)h_ctr + 16;
            for (int k = 0; k < 3; k++) t3[k] = t[k] + t[3 + k];
        } else {
            HIP_CHECK(hipEventRecord(t_end, stream));
            HIP_CHECK(hipMemcpyAsync(h_ctr + 8, st.stats, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
            read_unit_stats(t3);  // both statistics regions; synchronizes the stream
            examined = h_ctr[8];
        }
        // unit path: 16 B per row opened (offset pair), 4 B per interior edge, 4 B per
        // reverse entry, 4+4 B per request (root, target), 8 B per result word
        rs.unit_rows = t3[0];
        rs.unit_edges = t3[1];
        rs.unit_rev = t3[2];
        // v2 reads a 16 B edge record per edge and its row opens are the root/reverse
        // offset pairs only; v1 reads 4 B column entries and opens every frontier row
        rs.bytes_unit = 16 * rs.unit_rows + (use_v2 && !wave_u ? 16 : 4) * rs.unit_edges + 4 * rs.unit_rev +
                        8 * q.n + 8 * words;
        rs.rev_edges = examined + rs.unit_rev;
        rs.interior_edges += rs.unit_edges;
        // global path pull bytes: 16 per request row open (rev_off), 4 per reverse entry,
        // 8 per visited-word read, 8 per result word
        rs.bytes_pull = examined ? 16 * q.n + 4 * examined + 8 * examined + 8 * words : 0;
        rs.bytes_total = rs.bytes_unit + rs.bytes_push + rs.bytes_pull + 8 * 2 * rs.touched;
        float ms = 0;
        for (size_t i = 0; i < unit_ev.size(); i++) {
            HIP_CHECK(hipEventElapsedTime(&ms, unit_ev[i].first, unit_ev[i].second));
            rs.ms_unit += ms;
            if (i == 0) rs.main_ms = ms;
            if (i == 1 && use_bidi && bidi_cfg.lite == 3) rs.rest_ms = ms;
        }
        for (auto &p : push_ev) {
            HIP_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
            rs.ms_push += ms;
        }
        for (auto &p : pull_ev) {
            HIP_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
            rs.ms_pull += ms;
        }
        if (lean_call)
            ms = (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
        else
            HIP_CHECK(hipEventElapsedTime(&ms, t_begin, t_end));
        rs.ms_total = ms;
        last = rs;
        // no rest request: nothing wrote a flag word (and they were zero when it started)
        qq.flags_zero = label_resident && label_clean;
        if (stamps && use_units && !wave_u) report_stamps();
    }

    void ensure_io(uint64_t n) {
        if (io && n <= io_cap) return;
        delete io;
        io = nullptr;
        io_cap = std::max<uint64_t>((n + 63) / 64 * 64, 1 << 16);
        auto q = std::make_unique<ketogpu_queries>();
        q->d_roots = dalloc<uint32_t>(io_cap);
        q->d_targets = dalloc<uint32_t>(io_cap);
        q->d_allowed = dalloc<uint64_t>(io_cap / 64);
        q->d_flags = dalloc<uint64_t>(io_cap / 64);
        io = q.release();
    }

    // the device's view of host memory it can read in place (host_view), else nullptr
    const uint32_t *device_view(const uint32_t *p, bool query = true) {
        return (const uint32_t *)host_view(p, device, query);
    }

    void ensure_res(uint64_t n) {
        if (n <= res_cap) return;
        if (h_res) (void)hipHostFree(h_res);
        h_res = nullptr;
        res_cap = std::max<uint64_t>(n, 1 << 14);
        HIP_CHECK(hipHostMalloc((void **)&h_res, res_cap * 8, hipHostMallocDefault));
    }

    void check_bad(uint64_t first_bad) {
        if (first_bad != ~0ull)
            throw Error(KETOGPU_EINVAL, "request " + std::to_string(first_bad) + " has a node id outside the snapshot");
    }

    // SubjectIsAllowed over a batch held in host memory (SURVEY 8(d) "throughput timing":
    // requests H2D, traversal, result bits D2H).  Persistent HBM buffers, ids validated on
    // the device, and with the bidi plan a pipelined first stage (run_units, HostSrc): the
    // chunks' uploads overlap the traversal of the chunks before them, and the result copy
    // is enqueued ahead of the run's one host synchronization.  Host arrays allocated
    // with ketogpu_host_alloc (pinned) are copied by DMA at full PCIe rate.
    void check_host(const uint32_t *roots, const uint32_t *targets, uint64_t n, uint64_t *allowed, uint64_t *flagged) {
        HIP_CHECK(hipSetDevice(device));
        ensure_io(n);
        ketogpu_queries &q = *io;
        q.n = n;
        const uint64_t words = (n + 63) / 64;
        emit_req = EmitReq{};
        clear_bad = nullptr;
        const bool bidi_ok = n && use_units && !wave_u && (use_v2 || use_lite) && use_bidi && !(trials_left && n >= kTrialMin);
        // KETOGPU_PIPE_DMA=1: pinned requests are copied by DMA (copy engines) instead of
        // read in place by the device (CUs); an A/B knob
        static const bool dma = getenv("KETOGPU_PIPE_DMA") != nullptr;
        const bool big = n >= 2 * pipe_chunk;
        // the device's view of the request arrays: ketogpu_host_alloc buffers from the
        // registry; other pinned memory by a runtime query, asked for big batches only
        const uint32_t *dr = nullptr, *dt = nullptr;
        if (bidi_ok && !dma) {
            dr = device_view(roots, big);
            dt = dr ? device_view(targets, big) : nullptr;
        }
        const bool mapped = dr && dt;
        // host-batch first stage: pinned requests read in place by one launch (any size),
        // else the chunk pipeline for big batches
        const bool pipe = bidi_ok && ((mapped && pipe_direct) || big);
        if (!pipe) HIP_CHECK(hipMemsetAsync(d_bad, 0xFF, sizeof(unsigned long long), stream));
        if (!pipe) {
            if (n) {
                HIP_CHECK(hipMemcpyAsync(q.d_roots, roots, n * 4, hipMemcpyHostToDevice, stream));
                HIP_CHECK(hipMemcpyAsync(q.d_targets, targets, n * 4, hipMemcpyHostToDevice, stream));
                KLAUNCH(validate_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, q.d_roots, q.d_targets, n, g.Nx,
                        g.N, 0ull, d_bad);
            }
            run(q);
        } else {
            const HostSrc src{mapped ? dr : roots, mapped ? dt : targets, mapped};
            ensure_res(2 * words + 1);
            clear_bad = d_bad;  // reset by the run's clear launch
            // results, flags and the validation verdict in one launch with the statistics
            // result words straight into the caller's buffer when it is a ketogpu_host_alloc
            // buffer (no host copy after the call)
            uint64_t *direct_bits = allowed ? (uint64_t *)host_view(allowed, device, false) : nullptr;
            emit_req = EmitReq{q.d_allowed, flagged ? q.d_flags : nullptr, words, d_bad, h_res, direct_bits};
            run_once(q, &src, [&] {
                if (emit_req.out) {  // not taken by the bidi cascade's tail
                    KLAUNCH(emit_kernel, dim3((unsigned)std::min<uint64_t>(blocks_for(2 * words + 1), 256)),
                            dim3(kBlock), 0, stream, q.d_allowed, flagged ? q.d_flags : nullptr, words, d_bad, h_res,
                            direct_bits);
                    emit_req = EmitReq{};
                }
            });
            // the staged words were final unless requests went on to the global path
            if (!last.spilled_requests) {
                const uint64_t nf = flagged ? words : 0;
                if (allowed && !direct_bits) memcpy(allowed, h_res, words * 8);
                if (flagged) memcpy(flagged, h_res + words, words * 8);
                check_bad(h_res[words + nf]);
                return;
            }
        }
        HIP_CHECK(hipMemcpyAsync(h_ctr + 40, d_bad, 8, hipMemcpyDeviceToHost, stream));
        download(q, allowed, flagged);  // synchronizes
        check_bad(h_ctr[40]);
    }

    // validate = false: ids built by the library itself (ketogpu_check, dynamic roots)
    ketogpu_queries *upload(const uint32_t *roots, const uint32_t *targets, uint64_t n, bool validate = true) {
        HIP_CHECK(hipSetDevice(device));
        auto q = std::make_unique<ketogpu_queries>();
        q->n = n;
        uint64_t words = std::max<uint64_t>((n + 63) / 64, 1);
        q->d_roots = dalloc<uint32_t>(n);
        q->d_targets = dalloc<uint32_t>(n);
        q->d_allowed = dalloc<uint64_t>(words);
        q->d_flags = dalloc<uint64_t>(words);
        if (n) {
            HIP_CHECK(hipMemcpyAsync(q->d_roots, roots, n * 4, hipMemcpyHostToDevice, stream));
            HIP_CHECK(hipMemcpyAsync(q->d_targets, targets, n * 4, hipMemcpyHostToDevice, stream));
        }
        HIP_CHECK(hipMemsetAsync(q->d_allowed, 0, words * 8, stream));
        if (validate && n) {  // never launch on ids the graph does not have
            HIP_CHECK(hipMemsetAsync(d_bad, 0xFF, sizeof(unsigned long long), stream));
            KLAUNCH(validate_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, q->d_roots, q->d_targets, n, g.Nx,
                    g.N, 0ull, d_bad);
            HIP_CHECK(hipMemcpyAsync(h_ctr + 40, d_bad, 8, hipMemcpyDeviceToHost, stream));
        }
        HIP_CHECK(hipStreamSynchronize(stream));
        if (validate && n) check_bad(h_ctr[40]);
        return q.release();
    }

    void download(ketogpu_queries &q, uint64_t *allowed, uint64_t *flagged) {
        HIP_CHECK(hipSetDevice(device));
        uint64_t words = (q.n + 63) / 64;
        if (q.pending) {  // after this batch's queued call only (later queued calls keep running)
            HIP_CHECK(hipStreamWaitEvent(copy_stream, q.done_ev, 0));
            if (words && allowed)
                HIP_CHECK(hipMemcpyAsync(allowed, q.d_allowed, words * 8, hipMemcpyDeviceToHost, copy_stream));
            if (words && flagged)
                HIP_CHECK(hipMemcpyAsync(flagged, q.d_flags, words * 8, hipMemcpyDeviceToHost, copy_stream));
            HIP_CHECK(hipStreamSynchronize(copy_stream));
            q.pending = false;
            return;
        }
        drain_pipe();
        if (words && allowed)
            HIP_CHECK(hipMemcpyAsync(allowed, q.d_allowed, words * 8, hipMemcpyDeviceToHost, stream));
        if (words && flagged)
            HIP_CHECK(hipMemcpyAsync(flagged, q.d_flags, words * 8, hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
    }
};

// ------------------------------------------------------------------- C ABI
#define API_BEGIN try {
#define API_END                                                                                        \
    }                                                                                                  \
    catch (const Error &e) {                                                                           \
        set_last_error(e.what());                                                                      \
        return e.code;                                                                                 \
    }                                                                                                  \
    catch (const std::bad_alloc &) {                                                                   \
        set_last_error("out of host memory");                                                          \
        return KETOGPU_ENOMEM;                                                                         \
    }                                                                                                  \
    return KETOGPU_OK;

extern "C" {

int ketogpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ketogpu_engine_new(const ketogpu_snapshot *s, const ketogpu_engine_opts *opts, ketogpu_engine **out) {
    API_BEGIN
    if (!s || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto e = std::make_unique<ketogpu_engine>();
    const Snapshot &snap = *reinterpret_cast<const Snapshot *>(s);
    std::shared_lock<std::shared_mutex> rd(snap.mu);
    e->init(snap, opts);
    e->synced_version = snap.version;  // built from the current rows
    e->patch_pos = snap.patch_end();
    snap.reader_at(e.get(), e->patch_pos);
    e->snap_link = snap.link;
    {
        std::lock_guard<std::mutex> lk(snap.link->mu);
        snap.link->snap = &snap;
    }
    *out = e.release();
    API_END
}

void ketogpu_engine_free(ketogpu_engine *e) { delete e; }

int ketogpu_queries_upload(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                           ketogpu_queries **out) {
    API_BEGIN
    if (!e || !out || (n && (!roots || !targets))) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    e->sync();
    *out = e->upload(roots, targets, n);  // ids are validated on the device
    API_END
}

int ketogpu_queries_run(ketogpu_engine *e, ketogpu_queries *q) {
    API_BEGIN
    if (!e || !q) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    e->sync();
    e->run(*q);
    q->pending = false;  // (ran to completion)
    API_END
}

int ketogpu_queries_run_async(ketogpu_engine *e, ketogpu_queries *q, int *queued) {
    API_BEGIN
    if (!e || !q) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    e->pipelined_req = true;
    e->queued = false;
    try {
        e->sync();
    } catch (...) {
        e->pipelined_req = false;
        throw;
    }
    // calls rotate over kPipe streams: this call's first stage may run beside earlier calls'
    // dense passes (their counter sets and record regions differ, ketogpu_engine label_rest /
    // label_full)
    const unsigned si = e->use_label ? (unsigned)(e->label_calls % ketogpu_engine::kPipe) : 0u;
    if (si && !e->pipe_s[si]) HIP_CHECK(hipStreamCreateWithFlags(&e->pipe_s[si], hipStreamNonBlocking));
    hipStream_t sq = si ? e->pipe_s[si] : e->stream;
    bool elsewhere = false;  // the same batch queued on another stream: after it
    for (unsigned k = 0; k < ketogpu_engine::kPipe; k++) elsewhere |= k != si && e->pipe_q[k] == q;
    if (elsewhere && q->pending) HIP_CHECK(hipStreamWaitEvent(sq, q->done_ev, 0));
    if (si) std::swap(e->stream, e->pipe_s[si]);
    try {
        e->run(*q);
    } catch (...) {
        if (si) std::swap(e->stream, e->pipe_s[si]);
        e->pipelined_req = false;
        throw;
    }
    if (si) std::swap(e->stream, e->pipe_s[si]);
    if (e->queued) {
        if (!q->done_ev) HIP_CHECK(hipEventCreateWithFlags(&q->done_ev, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(q->done_ev, sq));
        q->pending = true;
        e->pipe_q[si] = q;
        e->pipe_used[si] = true;
    } else {
        e->pipe_q[si] = nullptr;  // (it ran to completion on its stream)
        q->pending = false;
    }
    e->pipelined_req = false;
    if (queued) *queued = e->queued ? 1 : 0;
    API_END
}

int ketogpu_engine_wait(ketogpu_engine *e) {
    API_BEGIN
    if (!e) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_CHECK(hipSetDevice(e->device));
    e->drain_pipe();
    HIP_CHECK(hipStreamSynchronize(e->stream));
    API_END
}

int ketogpu_queries_download(ketogpu_engine *e, const ketogpu_queries *q, uint64_t *allowed_bits,
                             uint64_t *flagged_bits) {
    API_BEGIN
    if (!e || !q) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    e->download(const_cast<ketogpu_queries &>(*q), allowed_bits, flagged_bits);
    API_END
}

void ketogpu_queries_free(ketogpu_queries *q) { delete q; }

int ketogpu_check_ids(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                      uint64_t *allowed_bits, uint64_t *flagged_bits) {
    API_BEGIN
    if (!e || (n && (!roots || !targets || !allowed_bits))) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    e->sync();
    e->check_host(roots, targets, n, allowed_bits, flagged_bits);
    API_END
}

int ketogpu_host_alloc(size_t bytes, void **out) {
    API_BEGIN
    if (!out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    const size_t n = std::max<size_t>(bytes, 1);
    // portable: pinned for every device of the process (a MultiEngine reads one batch
    // buffer from all of them); mapped: each device reads it in place through its own view
    HIP_CHECK(hipHostMalloc(out, n, hipHostMallocPortable | hipHostMallocMapped));
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    g_pinned[(uintptr_t)*out] = PinnedRange{n, {}};
    API_END
}

void ketogpu_host_free(void *p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned.erase((uintptr_t)p);
    }
    (void)hipHostFree(p);
}

int ketogpu_check(ketogpu_engine *e, const ketogpu_check_request *reqs, size_t n, uint8_t *allowed, int32_t *status) {
    API_BEGIN
    if (!e || (n && (!reqs || !allowed))) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    e->sync();
    const Snapshot &s = *e->snap;
    std::vector<uint32_t> roots(n, NONE), targets(n, NONE);
    // dynamic roots: wildcard queries with no snapshot node, materialized per batch
    std::vector<uint64_t> dio{0}, dfo{0};
    std::vector<uint32_t> dint, dfull, damb;
    std::vector<uint32_t> rows;
    std::vector<std::pair<size_t, RowRef>> dyn_rows;  // request -> materialized rows (host)
    std::vector<uint32_t> dyn_store;
    for (size_t i = 0; i < n; i++) {
        const ketogpu_check_request &r = reqs[i];
        if (status) status[i] = KETOGPU_OK;
        if (r.subject.kind != KETOGPU_SUBJECT_ID && r.subject.kind != KETOGPU_SUBJECT_SET) {
            if (status) status[i] = KETOGPU_EINVAL;  // ErrNilSubject (documented divergence)
            continue;
        }
        targets[i] = resolve_subject(s, r.subject);
        ResolvedRoot rr = resolve_root(s, sv(r.ns), sv(r.obj), sv(r.rel));
        if (rr.kind == ResolvedRoot::NODE) {
            roots[i] = rr.node;
        } else if (rr.kind == ResolvedRoot::DYNAMIC && targets[i] != NONE) {
            rows.clear();
            RowRef q = s.materialize(rr.any_ns, rr.ns, rr.obj, rr.any_obj, rr.rel, rr.any_rel, rows);
            if (!q.len) continue;
            uint32_t k = (uint32_t)(dio.size() - 1);
            roots[i] = kDynBase + k;
            RowRef keep = q;
            keep.off = dyn_store.size();
            dyn_store.insert(dyn_store.end(), rows.begin(), rows.begin() + q.len);
            dyn_rows.push_back({i, keep});
            std::vector<uint32_t> srt(rows.begin(), rows.begin() + q.len);
            std::sort(srt.begin(), srt.end());
            srt.erase(std::unique(srt.begin(), srt.end()), srt.end());
            uint32_t amb = 0;
            for (uint32_t u : srt) {
                dfull.push_back(u);
                if (u < s.Ni) dint.push_back(u);
                amb |= s.ambiguous[u];
            }
            damb.push_back(amb);
            dio.push_back(dint.size());
            dfo.push_back(dfull.size());
        }
    }
    std::unique_ptr<ketogpu_queries> q(e->upload(roots.data(), targets.data(), n, false));
    if (dio.size() > 1) {
        q->has_dyn = true;
        q->d_dyn_int_off = dupload(dio);
        q->d_dyn_full_off = dupload(dfo);
        q->d_dyn_int = dupload(dint);
        q->d_dyn_full = dupload(dfull);
        q->d_dyn_amb = dupload(damb);
    }
    e->run(*q);
    uint64_t words = (n + 63) / 64;
    std::vector<uint64_t> ab(words), fb(words);
    e->download(*q, ab.data(), fb.data());
    for (size_t i = 0; i < n; i++) allowed[i] = (ab[i >> 6] >> (i & 63)) & 1;
    // Requests that touched a Subject.String() key shared by two nodes (R4): the
    // reference's answer then depends on its DFS order; evaluate those sequentially.
    if (s.has_ambiguous) {
        for (size_t i = 0; i < n; i++) {
            if (!((fb[i >> 6] >> (i & 63)) & 1)) continue;
            if (roots[i] == NONE) continue;
            const uint32_t *rp;
            uint32_t rl;
            if (roots[i] >= kDynBase) {
                auto it = std::find_if(dyn_rows.begin(), dyn_rows.end(), [&](auto &p) { return p.first == i; });
                rp = dyn_store.data() + it->second.off;
                rl = it->second.len;
            } else {
                rp = s.row_ptr(roots[i]);
                rl = s.node_row[roots[i]].len;
            }
            allowed[i] = exact_check(s, rp, rl, reqs[i].subject, targets[i]) ? 1 : 0;
        }
    }
    API_END
}

int ketogpu_engine_sync(ketogpu_engine *e, double *ms, uint64_t *rows) {
    API_BEGIN
    if (!e) throw Error(KETOGPU_EINVAL, "null argument");
    const auto t0 = std::chrono::steady_clock::now();
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_CHECK(hipSetDevice(e->device));
    const uint64_t n = e->sync();
    if (rows) *rows = n;
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    API_END
}

int ketogpu_engine_label_heads(ketogpu_engine *e, int side, uint32_t *out, uint64_t capacity, uint64_t *words,
                               uint32_t *head_words) {
    API_BEGIN
    if (!e || !words || !head_words || side < 0 || side > 1) throw Error(KETOGPU_EINVAL, "bad argument");
    std::lock_guard<std::mutex> lk(e->mu);
    *words = e->use_label ? e->label_nwords[side] : 0;
    *head_words = e->use_label ? (side == 0 ? e->label_hs : e->label_hp) : 0;
    if (out && *words && capacity >= *words) {
        HIP_CHECK(hipSetDevice(e->device));
        HIP_CHECK(hipMemcpy(out, side == 0 ? e->lgraph.S : e->lgraph.P, *words * 4, hipMemcpyDeviceToHost));
    }
    API_END
}

int ketogpu_engine_check_graph(ketogpu_engine *e, uint64_t *mismatches) {
    API_BEGIN
    if (!e || !mismatches) throw Error(KETOGPU_EINVAL, "null argument");
    std::shared_lock<std::shared_mutex> rd(e->snap->mu);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_CHECK(hipSetDevice(e->device));
    e->sync();
    const Snapshot &s = *e->snap;
    uint64_t bad = 0;
    std::string first;
    auto note = [&](const char *what, size_t k, uint64_t got, uint64_t want) {
        if (first.empty())
            first = std::string(what) + " entry " + std::to_string(k) + ": device " + std::to_string(got) + ", host " +
                    std::to_string(want);
    };
    auto cmp_rows = [&](const uint32_t *dcol, const FRec *drec, const std::vector<uint32_t> &col, bool rev) {
        std::vector<uint32_t> c(col.size());
        if (!col.empty()) HIP_CHECK(hipMemcpy(c.data(), dcol, col.size() * 4, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < col.size(); k++)
            if (c[k] != col[k]) bad++, note(rev ? "reverse col" : "forward col", k, c[k], col[k]);
        if (!drec) return;
        std::vector<FRec> r(col.size());
        if (!col.empty()) HIP_CHECK(hipMemcpy(r.data(), drec, col.size() * sizeof(FRec), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < col.size(); k++) {
            const uint32_t u = col[k];
            const FRec want = rev ? (u < s.Ni ? FRec{u, ketogpu_engine::ideg(s, u), (uint32_t)s.rev_off[u], 0}
                                              : FRec{u, 0, 0, 0})
                                  : FRec{u, ketogpu_engine::fdeg(s, u), (uint32_t)s.fint_off[u], r[k].pad};
            if (r[k].node != want.node || r[k].deg != want.deg || r[k].begin != want.begin) {
                bad++;
                note(rev ? "reverse record (node<<32|deg)" : "forward record (node<<32|deg)", k,
                     (uint64_t)r[k].node << 32 | r[k].deg, (uint64_t)want.node << 32 | want.deg);
            }
        }
    };
    cmp_rows(e->g.fint_col, e->frec, s.fint_col, false);
    cmp_rows(e->g.rev_col, e->brec, s.rev_col, true);
    *mismatches = bad;
    set_last_error(first);
    API_END
}

int ketogpu_engine_set_events(ketogpu_engine *e, int every_kernel) {
    if (!e) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    std::lock_guard<std::mutex> lk(e->mu);
    e->light_events = !every_kernel;
    return KETOGPU_OK;
}

int ketogpu_engine_last_stats(const ketogpu_engine *e, ketogpu_run_stats *out) {
    if (!e || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    *out = e->last;
    return KETOGPU_OK;
}

}  // extern "C"
