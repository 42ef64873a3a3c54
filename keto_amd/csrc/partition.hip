// partition.hip — hash-partitioned traversal for graphs that do not fit one GPU
// (BASELINE.json config #5).
//
// A rank's partition is its shard (shard.cpp, loaded from the one ordered row stream by
// every rank): node v is owned by rank part_owner(v) (ids interleave the ranks inside the
// interior / expandable / other ranges, so owner and local index are arithmetic and no
// rank holds a per-node table of the whole graph).  A rank holds, for the nodes it owns:
// the forward interior rows and the 64-request traversal state of its expandable nodes,
// and the reverse rows of its nodes.  One round checks up to 64*W
// requests (W words of the multi-source bitmask BFS of SURVEY.md 8(a)):
//   begin      owned roots r seed (word, u, bit) for u in fint(r)
//   emit       outgoing records grouped by owner(u) into the caller's send buffer
//   [exchange] all-to-all of counts, then records (keto_amd/partition.py: RCCL)
//   apply      received masks OR'd into vis[word][u]; bits new to u enter the frontier
//   [all-reduce of the frontier size: stop at 0 — no depth cutoff, R2]
//   expand     the owned frontier's rows -> next outgoing records
//   pull_emit  for owned targets t: r in rev(t) is a direct hit, every interior v in
//              rev(t) becomes a query (request, v) for owner(v)
//   pull_answer  a query is a hit when vis[word][v] has the request's bit
//   end        this rank's hit bits; the answer is their OR over ranks
// The check formula is the one the single-GPU engines use: allowed(r, t)
// <=> r in rev(t) or rev(t) ∩ X(r) != {} with X(r) the interior closure of r.
// A round runs in one of two directions (ketogpu_part_begin_dir), the same steps:
//   forward    as above: the BFS grows X(r) from the roots' owners along forward interior
//              rows; the pull asks whether an interior v in rev(t) is in X(r)
//   backward   the BFS grows B(t) = interior nodes that reach t, seeded by the targets'
//              owners with the interior entries of rev(t) (r in rev(t) is a hit there),
//              along interior-predecessor rows; the pull sends (request, u) for u in
//              fint(r) from the roots' owners: u in B(t) <=> r reaches t in >= 2 edges.
// Which side is cheaper depends on the graph (RBAC: documents fan out to many groups, a
// user reaches few); keto_amd/partition.py times both and keeps the faster.
// Graphs with ambiguous Subject.String() keys (R4) are refused (the shard loader counts
// them): their exact re-evaluation needs the whole graph on one host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "device_util.hpp"
#include "ketogpu_internal.hpp"
#include "part_round.hpp"

using namespace ketogpu;
using namespace kdev;

namespace {

constexpr int kPB = 256;
constexpr int kPItems = 4;
constexpr int kPTile = kPB * kPItems;
// records per thread of part_apply_kernel (build knob for A/B)
#ifndef KETO_APPLY_ITEMS
#define KETO_APPLY_ITEMS 4
#endif
constexpr int kAItems = KETO_APPLY_ITEMS;
constexpr int kATile = kPB * kAItems;
constexpr uint32_t kMaxWorld = 64;

// Owner of global node id v (the shard layout, shard.cpp): inside each class range —
// interior [0, Ni), other expandable [Ni, Nx), never expanded [Nx, N) — ids interleave
// the ranks.
__host__ __device__ __forceinline__ uint32_t part_owner(uint32_t v, uint32_t Ni, uint32_t Nx, uint32_t world) {
    const uint32_t base = v < Ni ? 0u : v < Nx ? Ni : Nx;
    return (v - base) % world;
}

struct PartDev {
    uint32_t world, rank, Ni, Nx, N;  // global layout
    uint32_t Nil, Nxl, Nl;            // this rank's class bounds: owned interior | expandable | all
    const uint64_t *lf_off;  // [Nxl + 1] forward interior rows of owned expandable nodes
    const uint32_t *lf_col;  //           (global node ids)
    const uint64_t *lr_off;  // [Nl + 1] reverse rows of owned nodes (global ids, sorted)
    const uint32_t *lr_col;
    const uint64_t *lb_off;  // [Nil + 1] interior predecessors of owned interior nodes (backward rows)
    const uint32_t *lb_col;
    uint32_t dir;            // round direction: 0 forward, 1 backward
    uint64_t *vis, *nxt;     // [W][Nil] visited bits of the round's requests, new bits of the level
    uint64_t *fe_key, *fe_pre, *fe_mask;
    uint64_t fe_cap;
    uint64_t *touch;
    uint64_t touch_cap;
    ketogpu_record *obuf;    // outgoing records of the current step (unordered)
    uint64_t ocap;
    unsigned long long *ctr;  // [0..1] frontier counters (ping-pong), [2] touch, [3] obuf, [4..5] overflow
    unsigned int *overflow;   // bit 0 list/buffer overflow, bit 1 misrouted record, bit 2 invalid request id
    uint64_t *allowed;        // this rank's hit bits of the round
    const uint32_t *roots, *targets;
    uint64_t n;
};

__device__ __forceinline__ uint32_t p_owner(const PartDev &P, uint32_t v) { return part_owner(v, P.Ni, P.Nx, P.world); }

// local index of node v if this rank owns it (NONE otherwise, and for ids of the layout's
// unused slots)
__device__ __forceinline__ uint32_t p_local(const PartDev &P, uint32_t v) {
    if (v >= P.N || p_owner(P, v) != P.rank) return KETOGPU_NODE_NONE;
    uint32_t l, lim;
    if (v < P.Ni) {
        l = v / P.world;
        lim = P.Nil;
    } else if (v < P.Nx) {
        l = P.Nil + (v - P.Ni) / P.world;
        lim = P.Nxl;
    } else {
        l = P.Nxl + (v - P.Nx) / P.world;
        lim = P.Nl;
    }
    return l < lim ? l : KETOGPU_NODE_NONE;
}

__device__ __forceinline__ void put_rec(uint64_t idx, uint32_t a, uint32_t b, uint64_t m, const PartDev &P) {
    if (idx < P.ocap)
        P.obuf[idx] = ketogpu_record{a, b, m};
    else
        atomicOr(P.overflow, 1u);
}

// One wave writes its lanes' row slices [b, b + len) as consecutive records (lane 0's
// first): each output index finds its lane by a binary search over the wave's prefix in
// LDS, so consecutive lanes write consecutive records and read consecutive row entries
// (a lane looping over its own row wrote one record per lane per instruction, 64 lines
// apart: seed 0.25 ms and pull_emit 0.45 ms per 10^6 requests).  Record of lane j's k-th
// entry: pull = false (word, node, bit) of request i_j; pull = true (request i_j, node, 0).
// Every thread of the block calls it (two block barriers).
__device__ __forceinline__ void wave_emit(uint64_t b, uint64_t len, const uint32_t *col, bool pull,
                                          const PartDev &P) {
    __shared__ uint64_t s_pre[kPB / 64][65];
    __shared__ uint64_t s_b[kPB / 64][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan(len, lane);
    const uint64_t total = __shfl(incl, 63, 64);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(&P.ctr[3], (unsigned long long)total);
    base = __shfl(base, 63, 64);
    s_pre[wv][lane] = incl - len;
    s_b[wv][lane] = b;
    if (lane == 0) s_pre[wv][64] = total;
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * kPB + (uint64_t)wv * 64;
    for (uint64_t o = lane; o < total; o += 64) {
        int lo = 0, hi = 64;  // the last lane j with s_pre[j] <= o owns o (empty lanes never win)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_pre[wv][mid] <= o)
                lo = mid;
            else
                hi = mid;
        }
        const uint64_t i = i0 + (uint64_t)lo;
        const uint32_t v = col[s_b[wv][lo] + (o - s_pre[wv][lo])];
        if (pull)
            put_rec(base + o, (uint32_t)i, v, 0, P);
        else
            put_rec(base + o, (uint32_t)(i >> 6), v, 1ull << (i & 63), P);
    }
    __syncthreads();
}

// first index of the sorted row [b, e) whose entry is >= key
__device__ __forceinline__ uint64_t row_lower_bound(const uint32_t *col, uint64_t b, uint64_t e, uint32_t key) {
    while (b < e) {
        const uint64_t mid = (b + e) >> 1;
        if (col[mid] < key)
            b = mid + 1;
        else
            e = mid;
    }
    return b;
}

// forward: owned roots, (word, u, bit) for every interior successor u.  Backward: owned
// targets, r in rev(t) is a hit, (word, v, bit) for every interior v in rev(t).
__global__ __launch_bounds__(kPB) void part_seed_kernel(PartDev P) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    uint64_t b = 0, e = 0;
    // ids outside the snapshot: the round fails with KETOGPU_EINVAL at the first emit (bit 2)
    if (i < P.n && ((P.roots[i] != KETOGPU_NODE_NONE && P.roots[i] >= P.Nx) ||
                    (P.targets[i] != KETOGPU_NODE_NONE && P.targets[i] >= P.N)))
        atomicOr(P.overflow, 4u);
    if (P.dir) {
        uint32_t r = KETOGPU_NODE_NONE;
        if (i < P.n) {
            const uint32_t t = P.targets[i];
            r = P.roots[i];
            if (t != KETOGPU_NODE_NONE && r != KETOGPU_NODE_NONE && r < P.Nx && t < P.N) {
                const uint32_t lt = p_local(P, t);
                if (lt != KETOGPU_NODE_NONE) {
                    b = P.lr_off[lt];
                    e = P.lr_off[lt + 1];
                }
            }
        }
        // rows are sorted, interior ids first: r in rev(t) by binary search, the interior
        // prefix seeds the BFS
        bool hit = false;
        if (b < e) {
            const uint64_t h = row_lower_bound(P.lr_col, b, e, r);
            hit = h < e && P.lr_col[h] == r;
            e = hit ? b : row_lower_bound(P.lr_col, b, e, P.Ni);
        }
        if (hit) atomicOr((unsigned long long *)&P.allowed[i >> 6], 1ull << (i & 63));
        wave_emit(b, e - b, P.lr_col, false, P);
        return;
    }
    if (i < P.n) {
        uint32_t r = P.roots[i], t = P.targets[i];
        if (r != KETOGPU_NODE_NONE && t != KETOGPU_NODE_NONE && r < P.Nx) {
            uint32_t l = p_local(P, r);
            if (l != KETOGPU_NODE_NONE) {
                b = P.lf_off[l];
                e = P.lf_off[l + 1];
            }
        }
    }
    wave_emit(b, e - b, P.lf_col, false, P);
}

// load-balanced expansion of frontier entries [ent_begin, ent_begin + ent_count)
// (row-length prefix in fe_pre) into outgoing records
__global__ __launch_bounds__(kPB) void part_expand_kernel(PartDev P, uint64_t ent_begin, uint64_t ent_count,
                                                          uint64_t total_edges) {
    __shared__ uint64_t s_pre[kPTile + 1];
    __shared__ uint64_t s_first, s_count;
    __shared__ unsigned long long s_out;  // the tile's records: one reservation per tile
    const int lane = threadIdx.x & 63;
    const uint64_t *pre = P.fe_pre + ent_begin;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kPTile; t0 < total_edges; t0 += (uint64_t)gridDim.x * kPTile) {
        const uint64_t t1 = t0 + kPTile < total_edges ? t0 + kPTile : total_edges;
        if (threadIdx.x < 64) {
            uint64_t i0 = wave_upper_bound(pre, ent_count, t0, lane) - 1;
            uint64_t i1 = wave_upper_bound(pre, ent_count, t1 - 1, lane) - 1;
            if (lane == 0) {
                s_first = i0;
                s_count = i1 - i0 + 1;
                s_out = atomicAdd(&P.ctr[3], (unsigned long long)(t1 - t0));
            }
        }
        __syncthreads();
        const uint64_t first = s_first, count = s_count;
        for (uint64_t j = threadIdx.x; j <= count; j += kPB)
            s_pre[j] = (first + j < ent_count) ? pre[first + j] : total_edges;
        __syncthreads();
#pragma unroll 1
        for (int it = 0; it < kPItems; it++) {
            const uint64_t e = t0 + (uint64_t)it * kPB + threadIdx.x;
            bool want = e < t1;
            uint32_t w = 0, u = 0;
            uint64_t m = 0;
            if (want) {
                uint64_t lo = 0, hi = count;  // entry j: s_pre[j] <= e < s_pre[j+1]
                while (hi - lo > 1) {
                    uint64_t mid = (lo + hi) >> 1;
                    if (s_pre[mid] <= e)
                        lo = mid;
                    else
                        hi = mid;
                }
                const uint64_t ent = ent_begin + first + lo;
                const uint64_t k = P.fe_key[ent];
                w = (uint32_t)(k >> 32);
                const uint32_t l = (uint32_t)k;
                m = P.fe_mask[ent];
                u = P.dir ? P.lb_col[P.lb_off[l] + (e - s_pre[lo])] : P.lf_col[P.lf_off[l] + (e - s_pre[lo])];
                put_rec(s_out + (e - t0), w, u, m, P);
            }
        }
        __syncthreads();
    }
}

// per-destination record counts (LDS histogram, one global atomic per rank per block)
__global__ __launch_bounds__(kPB) void part_count_kernel(PartDev P, const ketogpu_record *rec, uint64_t n,
                                                         unsigned long long *counts) {
    __shared__ uint32_t h[kMaxWorld];
    if (threadIdx.x < kMaxWorld) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kPB)
        atomicAdd(&h[p_owner(P, rec[i].b)], 1u);
    __syncthreads();
    if (threadIdx.x < P.world && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// records -> out grouped by destination (cursor[g] starts at the group's offset); each
// block reserves its share of every group once per 256-record tile
__global__ __launch_bounds__(kPB) void part_scatter_kernel(PartDev P, const ketogpu_record *rec, uint64_t n,
                                                           unsigned long long *cursor, ketogpu_record *out) {
    const uint32_t world = P.world;
    __shared__ uint32_t h[kMaxWorld];
    __shared__ unsigned long long base[kMaxWorld];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kPB; t0 < n; t0 += (uint64_t)gridDim.x * kPB) {
        if (threadIdx.x < kMaxWorld) h[threadIdx.x] = 0;
        __syncthreads();
        const uint64_t i = t0 + threadIdx.x;
        const bool have = i < n;
        ketogpu_record r{0, 0, 0};
        uint32_t o = 0, pos = 0;
        if (have) {
            r = rec[i];
            o = p_owner(P, r.b);
            pos = atomicAdd(&h[o], 1u);
        }
        __syncthreads();
        if (threadIdx.x < world && h[threadIdx.x])
            base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]);
        __syncthreads();
        if (have) out[base[o] + pos] = r;
        __syncthreads();
    }
}

// KETO_APPLY_READ=1 (default): apply reads vis before its atomic OR and skips records
// that bring no new bit; 0: every record goes straight to the atomic (one dependent
// access less per record, one atomic more per redundant record)
#ifndef KETO_APPLY_READ
#define KETO_APPLY_READ 1
#endif

// received (word, u, mask): OR into the owned state, new bits enter the next frontier:
// they are ORed into nxt[word][u] and the record that finds nxt empty appends the entry,
// so a (word, u) is expanded once per level with all its new bits (the gather pass copies
// nxt into the list).  Appending every record's new bits as its own entry instead (no nxt,
// no gather) measured 0.33 ms faster per 10^6 config #5 requests but lets the entries of
// one (word, u) multiply along paths that split and merge again (up to 64 per level):
// rounds of one word overflowed small buffers that the deduplicated form fits.
// A block takes a tile of kPTile records (kPItems per thread) and makes ONE reservation
// on the packed frontier counter (count << kCntShift | row-length prefix) and one on the
// touch counter per tile: a reservation per wave serialised on the shared counter
// (690 us per level of ~3M records on config #2).
__global__ __launch_bounds__(kPB) void part_apply_kernel(PartDev P, const ketogpu_record *rec, uint64_t n,
                                                         uint64_t out_base, unsigned long long *out_ctr) {
    __shared__ uint64_t s_wsum[kPB / 64][2];  // per wave: packed append total, touch count
    __shared__ unsigned long long s_base[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kATile; t0 < n; t0 += (uint64_t)gridDim.x * kATile) {
        uint64_t key[kAItems], deg[kAItems];
        uint32_t app = 0, touched = 0;  // bit it: item it appends / is a vis-only entry
        uint64_t val = 0, tcnt = 0;
#pragma unroll
        for (int it = 0; it < kAItems; it++) {
            const uint64_t i = t0 + (uint64_t)it * kPB + threadIdx.x;
            key[it] = 0;
            deg[it] = 0;
            if (i >= n) continue;
            const ketogpu_record r = rec[i];
            const uint32_t l = p_local(P, r.b);
            if (l >= P.Nil) {
                atomicOr(P.overflow, 2u);  // not an interior node of this rank
                continue;
            }
            const size_t slot = (size_t)r.a * P.Nil + l;
#if KETO_APPLY_READ
            const uint64_t nw = r.m & ~P.vis[slot];  // skip the atomic when no bit is new
            if (!nw) continue;
#else
            const uint64_t nw = r.m;
#endif
            const uint64_t old = atomicOr((unsigned long long *)&P.vis[slot], (unsigned long long)nw);
            const uint64_t newly = nw & ~old;
            if (!newly) continue;
            key[it] = ((uint64_t)r.a << 32) | l;
            const uint64_t d = P.dir ? P.lb_off[l + 1] - P.lb_off[l] : P.lf_off[l + 1] - P.lf_off[l];
            if (d) {
                const uint64_t o2 = atomicOr((unsigned long long *)&P.nxt[slot], (unsigned long long)newly);
                if (!o2) {
                    app |= 1u << it;
                    deg[it] = d;
                    val += (1ull << kCntShift) | d;
                }
            } else if (!old) {
                touched |= 1u << it;  // vis-only entry: recorded once for the reset
                tcnt++;
            }
        }
        const uint64_t incl = wave_incl_scan(val, lane), tincl = wave_incl_scan(tcnt, lane);
        if (lane == 63) {
            s_wsum[wv][0] = incl;
            s_wsum[wv][1] = tincl;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t tot = 0, ttot = 0;
            for (int k = 0; k < kPB / 64; k++) tot += s_wsum[k][0], ttot += s_wsum[k][1];
            unsigned long long b0 = 0, b1 = 0;
            if (tot) {
                b0 = atomicAdd(out_ctr, (unsigned long long)tot);
                // a row-length prefix that carries into the count field corrupts both: flag it
                if ((b0 & kPreMask) + (tot & kPreMask) > kPreMask) atomicOr(P.overflow, 1u);
            }
            if (ttot) b1 = atomicAdd(&P.ctr[2], (unsigned long long)ttot);
            s_base[0] = b0;
            s_base[1] = b1;
        }
        __syncthreads();
        uint64_t pos = s_base[0] + incl - val, tpos = s_base[1] + tincl - tcnt;
        for (int k = 0; k < wv; k++) pos += s_wsum[k][0], tpos += s_wsum[k][1];
#pragma unroll
        for (int it = 0; it < kAItems; it++) {
            if ((app >> it) & 1u) {
                const uint64_t idx = out_base + (pos >> kCntShift);
                if (idx < P.fe_cap) {
                    P.fe_key[idx] = key[it];
                    P.fe_pre[idx] = pos & kPreMask;
                } else {
                    atomicOr(P.overflow, 1u);
                }
                pos += (1ull << kCntShift) | deg[it];
            }
            if ((touched >> it) & 1u) {
                if (tpos < P.touch_cap)
                    P.touch[tpos] = key[it];
                else
                    atomicOr(P.overflow, 1u);
                tpos++;
            }
        }
        __syncthreads();  // s_wsum / s_base are reused by the next tile
    }
}

// forward: owned targets, direct hits (r in rev(t)) and queries (request, interior v in
// rev(t)).  Backward: owned roots, queries (request, u) for u in fint(r).
// next level's masks: nxt -> entry list, nxt cleared
__global__ __launch_bounds__(kPB) void part_gather_kernel(PartDev P, uint64_t b, uint64_t e) {
    const uint64_t i = b + (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= e) return;
    const uint64_t k = P.fe_key[i];
    const size_t slot = (size_t)(k >> 32) * P.Nil + (uint32_t)k;
    P.fe_mask[i] = P.nxt[slot];
    P.nxt[slot] = 0;
}

__global__ __launch_bounds__(kPB) void part_pull_emit_kernel(PartDev P) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    uint64_t b = 0, e = 0;
    uint32_t r = KETOGPU_NODE_NONE;
    if (P.dir) {
        if (i < P.n) {
            const uint32_t t = P.targets[i];
            r = P.roots[i];
            if (t != KETOGPU_NODE_NONE && r != KETOGPU_NODE_NONE && r < P.Nx && t < P.N) {
                const uint32_t l = p_local(P, r);
                if (l != KETOGPU_NODE_NONE) {
                    b = P.lf_off[l];
                    e = P.lf_off[l + 1];
                }
            }
        }
        wave_emit(b, e - b, P.lf_col, true, P);
        return;
    }
    if (i < P.n) {
        const uint32_t t = P.targets[i];
        r = P.roots[i];
        if (t != KETOGPU_NODE_NONE && r != KETOGPU_NODE_NONE && r < P.Nx && t < P.N) {
            const uint32_t lt = p_local(P, t);
            if (lt != KETOGPU_NODE_NONE) {
                b = P.lr_off[lt];
                e = P.lr_off[lt + 1];
            }
        }
    }
    bool hit = false;
    if (b < e) {  // sorted row: r in rev(t) by binary search, queries for the interior prefix
        const uint64_t h = row_lower_bound(P.lr_col, b, e, r);
        hit = h < e && P.lr_col[h] == r;
        e = hit ? b : row_lower_bound(P.lr_col, b, e, P.Ni);
    }
    if (hit) atomicOr((unsigned long long *)&P.allowed[i >> 6], 1ull << (i & 63));
    wave_emit(b, e - b, P.lr_col, true, P);
}

__global__ __launch_bounds__(kPB) void part_pull_answer_kernel(PartDev P, const ketogpu_record *rec, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= n) return;
    const ketogpu_record r = rec[i];
    const uint32_t l = p_local(P, r.b);
    if (l >= P.Nil || r.a >= P.n) {
        atomicOr(P.overflow, 2u);
        return;
    }
    if ((P.vis[(size_t)(r.a >> 6) * P.Nil + l] >> (r.a & 63)) & 1ull)
        atomicOr((unsigned long long *)&P.allowed[r.a >> 6], 1ull << (r.a & 63));
}

__global__ __launch_bounds__(kPB) void part_reset_kernel(uint64_t *vis, uint32_t Nil, const uint64_t *keys, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kPB + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    vis[(size_t)(k >> 32) * Nil + (uint32_t)k] = 0;
}

inline unsigned pblocks(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + kPB - 1) / kPB); }

#define PHIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define KLAUNCH(...)                                 \
    do {                                             \
        hipLaunchKernelGGL(__VA_ARGS__);             \
        PHIP(hipGetLastError());                     \
    } while (0)

template <class T>
T *palloc(size_t n) {
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) throw Error(KETOGPU_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return (T *)p;
}

}  // namespace

struct ketogpu_part {
    int device = 0;
    uint32_t rank = 0, world = 1;
    hipStream_t stream = nullptr;
    std::mutex mu;
    PartDev P{};
    std::vector<void *> owned;
    uint64_t W = 1;                  // words per round
    uint32_t *d_roots = nullptr, *d_targets = nullptr;
    unsigned long long *d_counts = nullptr, *d_cursor = nullptr;
    unsigned long long *h = nullptr;  // pinned: counters and counts
    // frontier bookkeeping of the round
    uint64_t lb = 0, cnt = 0, edges = 0;
    int cur = 0;
    bool dirty = false;  // state may hold bits a sparse reset does not know about
    ketogpu_part_stats stats{};
    // Two state buffers (vis + the entry keys and touch list the sparse reset reads): a
    // round runs on buffer vb while the previous round's buffer is cleared on rstream, so
    // the reset (0.62 ms per 10^6 config #2 requests, random 8-B stores) overlaps the next
    // round instead of ending every round; begin() makes `stream` wait for its buffer.
    uint64_t *vis_buf[2] = {nullptr, nullptr}, *key_buf[2] = {nullptr, nullptr}, *touch_buf[2] = {nullptr, nullptr};
    int vb = 0;
    hipStream_t rstream = nullptr;
    hipEvent_t clean_ev[2] = {nullptr, nullptr}, done_ev = nullptr;
    bool clean_pending[2] = {false, false};
    void use_buffer(int b) {
        vb = b;
        P.vis = vis_buf[b];
        P.fe_key = key_buf[b];
        P.touch = touch_buf[b];
    }
    // the current buffer's clear (if one is in flight) before `stream` touches it
    void wait_clean() {
        if (clean_pending[vb]) PHIP(hipStreamWaitEvent(stream, clean_ev[vb], 0));
        clean_pending[vb] = false;
    }
    // measurement pass (ketogpu_part_set_timing): event pairs per launch, resolved at the
    // next host synchronization
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Pending {
        int fam;
        hipEvent_t a, b;
    };
    std::vector<Pending> pend;

    hipEvent_t ev() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e;
            PHIP(hipEventCreate(&e));
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }
    // bracket one launch (fam: KETOGPU_PART_K_*) with events while timing; bytes always
    template <class F>
    void timed(int fam, uint64_t bytes, F &&launch, hipStream_t on = nullptr) {
        stats.bytes[fam] += bytes;
        if (!timing) {
            launch();
            return;
        }
        if (!on) on = stream;
        hipEvent_t a = ev(), b = ev();
        PHIP(hipEventRecord(a, on));
        launch();
        PHIP(hipEventRecord(b, on));
        pend.push_back({fam, a, b});
    }
    // after a stream synchronization: fold the completed launches' times into the stats
    // (launches on rstream may still run: their end events are waited for)
    void resolve_timing() {
        for (const Pending &x : pend) {
            float ms = 0;
            PHIP(hipEventSynchronize(x.b));
            PHIP(hipEventElapsedTime(&ms, x.a, x.b));
            stats.ms[x.fam] += ms;
            stats.launches[x.fam]++;
        }
        pend.clear();
        ev_used = 0;
    }

    ~ketogpu_part() {
        if (stream) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(stream);
        }
        if (rstream) (void)hipStreamSynchronize(rstream);
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        for (auto e : clean_ev)
            if (e) (void)hipEventDestroy(e);
        if (done_ev) (void)hipEventDestroy(done_ev);
        if (rstream) (void)hipStreamDestroy(rstream);
        for (void *p : owned) (void)hipFree(p);
        if (h) (void)hipHostFree(h);
        if (stream) (void)hipStreamDestroy(stream);
    }

    template <class T>
    T *own(T *p) {
        owned.push_back((void *)p);
        return p;
    }
    template <class T>
    T *upload(const std::vector<T> &v) {
        T *p = own(palloc<T>(v.size()));
        if (!v.empty()) PHIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        return p;
    }

    void init(const ketogpu_shard *sh, const ketogpu_part_opts &o) {
        ketogpu_shard_graph v{};
        {
            const int rc = ketogpu_shard_view(sh, &v);
            if (rc) throw Error(rc, ketogpu_last_error());
        }
        if (o.world < 1 || (uint32_t)o.world > kMaxWorld || o.rank < 0 || o.rank >= o.world)
            throw Error(KETOGPU_EINVAL, "partition: need 0 <= rank < world <= 64");
        if ((uint32_t)o.rank != v.rank || (uint32_t)o.world != v.world)
            throw Error(KETOGPU_EINVAL, "partition: rank/world differ from the shard's");
        ketogpu_shard_stats ss{};
        if (ketogpu_shard_stats_get(sh, &ss) == KETOGPU_OK && ss.ambiguous_keys)
            throw Error(KETOGPU_EINVAL, "partition: the graph has ambiguous Subject.String() keys (R4)");
        device = o.device;
        rank = (uint32_t)o.rank;
        world = (uint32_t)o.world;
        int ndev = 0;
        PHIP(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw Error(KETOGPU_EDEVICE, "no such HIP device");
        PHIP(hipSetDevice(device));
        PHIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        PHIP(hipStreamCreateWithFlags(&rstream, hipStreamNonBlocking));
        for (auto &e : clean_ev) PHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        PHIP(hipEventCreateWithFlags(&done_ev, hipEventDisableTiming));
        auto upv = [&](const auto *p, size_t n) {
            using T = std::remove_const_t<std::remove_pointer_t<decltype(p)>>;
            return upload(std::vector<T>(p, p + n));
        };
        P.world = world;
        P.rank = rank;
        P.Ni = v.num_interior;
        P.Nx = v.num_expandable;
        P.N = v.num_nodes;
        P.Nil = v.owned_interior;
        P.Nxl = v.owned_expandable;
        P.Nl = v.owned_nodes;
        P.lf_off = upv(v.lf_off, (size_t)v.owned_expandable + 1);
        P.lf_col = upv(v.lf_col, (size_t)v.lf_off[v.owned_expandable]);
        P.lr_off = upv(v.lr_off, (size_t)v.owned_nodes + 1);
        P.lr_col = upv(v.lr_col, (size_t)v.lr_off[v.owned_nodes]);
        P.lb_off = upv(v.lb_off, (size_t)v.owned_interior + 1);
        P.lb_col = upv(v.lb_col, (size_t)v.lb_off[v.owned_interior]);
        stats.owned_interior = v.owned_interior;
        stats.owned_expandable = v.owned_expandable;
        stats.owned_forward_edges = v.lf_off[v.owned_expandable];
        stats.owned_reverse_edges = v.lr_off[v.owned_nodes];
        const uint32_t Nil = v.owned_interior;

        size_t free_b = 0, total_b = 0;
        PHIP(hipMemGetInfo(&free_b, &total_b));
        uint64_t budget = o.state_budget_bytes ? o.state_budget_bytes : std::min<uint64_t>(free_b / 4, 64ull << 30);
        budget = std::min<uint64_t>(budget, (uint64_t)free_b / 2);
        uint64_t lists = budget / 4;
        // per entry: key, prefix, mask, touch + the second buffer's key and touch
        P.fe_cap = std::min<uint64_t>(std::max<uint64_t>(lists / 48, 1 << 16), kMaxListEntries);
        P.touch_cap = P.fe_cap;
        P.ocap = o.record_capacity ? o.record_capacity : std::max<uint64_t>(lists / 16, 1 << 16);
        // 24 B per (word, node): the two vis buffers and nxt
        W = std::max<uint64_t>(1, (budget - std::min(budget, lists + P.ocap * 16)) / (24ull * std::max<uint32_t>(Nil, 1)));
        if (o.max_words_per_round) W = std::min<uint64_t>(W, o.max_words_per_round);
        W = std::max<uint64_t>(1, std::min<uint64_t>(W, 1u << 16));
        // Not bounded by fe_cap / (Nil + 64) (the worst case of one (word, node) entry per
        // owned node and word): that bound held config #2 to 2,680 words, six host-driven
        // rounds per 10^6 requests, while its searches touch ~12 nodes per request.  A level
        // whose entries exceed fe_cap (< 2^28, so the packed count cannot wrap unflagged:
        // device_util.hpp) or whose records exceed ocap sets the overflow flag; every rank
        // then aborts the round and retries it with half the requests (PartitionedEngine).
        const size_t state = (size_t)W * std::max<uint32_t>(Nil, 1);
        for (int b = 0; b < 2; b++) {
            vis_buf[b] = own(palloc<uint64_t>(state));
            PHIP(hipMemsetAsync(vis_buf[b], 0, state * 8, stream));
            key_buf[b] = own(palloc<uint64_t>(P.fe_cap));
            touch_buf[b] = own(palloc<uint64_t>(P.touch_cap));
        }
        use_buffer(0);
        P.nxt = own(palloc<uint64_t>(state));  // all zero between levels (the gather clears it)
        PHIP(hipMemsetAsync(P.nxt, 0, state * 8, stream));
        P.fe_pre = own(palloc<uint64_t>(P.fe_cap));
        P.fe_mask = own(palloc<uint64_t>(P.fe_cap));
        P.obuf = own(palloc<ketogpu_record>(P.ocap));
        P.ctr = own(palloc<unsigned long long>(8));
        P.overflow = (unsigned int *)(P.ctr + 4);  // in the counter block: one copy reads both
        P.allowed = own(palloc<uint64_t>(W));
        d_roots = own(palloc<uint32_t>(W * 64));
        d_targets = own(palloc<uint32_t>(W * 64));
        d_counts = own(palloc<unsigned long long>(kMaxWorld));
        d_cursor = own(palloc<unsigned long long>(kMaxWorld));
        PHIP(hipHostMalloc((void **)&h, (16 + 2 * kMaxWorld) * sizeof(unsigned long long), hipHostMallocDefault));
        P.roots = d_roots;
        P.targets = d_targets;
        PHIP(hipStreamSynchronize(stream));
    }

    void read_ctr() {
        // ctr[0..3] and the overflow flags (ctr[4], low word) in one copy
        PHIP(hipMemcpyAsync(h, P.ctr, 5 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
        PHIP(hipStreamSynchronize(stream));
        if (timing) resolve_timing();
    }
    uint32_t overflow_bits() const { return (uint32_t)h[4]; }

    void begin(const uint32_t *roots, const uint32_t *targets, uint64_t n, int dir) {
        if (dir != KETOGPU_PART_FORWARD && dir != KETOGPU_PART_BACKWARD)
            throw Error(KETOGPU_EINVAL, "partition: direction must be KETOGPU_PART_FORWARD or _BACKWARD");
        if (dirty) reset(true);
        wait_clean();
        P.dir = (uint32_t)dir;
        if (n > W * 64) throw Error(KETOGPU_EINVAL, "partition: more requests than one round holds");
        // ids are validated by the seed kernel (a host loop over 10^6 requests cost ~0.5 ms
        // per round); an invalid id fails the round's first emit with KETOGPU_EINVAL
        P.n = n;
        dirty = true;
        if (n) {
            PHIP(hipMemcpyAsync(d_roots, roots, n * 4, hipMemcpyHostToDevice, stream));
            PHIP(hipMemcpyAsync(d_targets, targets, n * 4, hipMemcpyHostToDevice, stream));
        }
        PHIP(hipMemsetAsync(P.ctr, 0, 8 * sizeof(unsigned long long), stream));
        PHIP(hipMemsetAsync(P.allowed, 0, W * 8, stream));
        lb = cnt = edges = 0;
        cur = 0;
        timed(KETOGPU_PART_K_SEED, 16 * n, [&] { KLAUNCH(part_seed_kernel, dim3(pblocks(n)), dim3(kPB), 0, stream, P); });
        PHIP(hipGetLastError());
        stats.rounds++;
    }

    // bucket obuf by destination into send; returns KETOGPU_ENOMEM on overflow
    int pack(ketogpu_record *send, uint64_t capacity, uint64_t *counts) {
        read_ctr();
        const uint64_t n = h[3];
        if (overflow_bits() || n > capacity) {
            for (uint32_t g = 0; g < world; g++) counts[g] = 0;
            return overflow_bits() & 4u ? KETOGPU_EINVAL : KETOGPU_ENOMEM;
        }
        if (n && world == 1 && !exchange_pack) {  // one destination: the records are already grouped
            // no copy: the caller hands `send` straight back to apply (its own records),
            // which then reads them where the kernels wrote them (obuf_send, apply)
            counts[0] = n;
            obuf_send = send;
            obuf_n = n;
        } else if (n) {
            PHIP(hipMemsetAsync(d_counts, 0, world * sizeof(unsigned long long), stream));
            unsigned grid = (unsigned)std::min<uint64_t>(pblocks(n), 2048);
            timed(KETOGPU_PART_K_PACK, 16 * n,
                  [&] { KLAUNCH(part_count_kernel, dim3(grid), dim3(kPB), 0, stream, P, P.obuf, n, d_counts); });
            PHIP(hipMemcpyAsync(h + 16, d_counts, world * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
            PHIP(hipStreamSynchronize(stream));
            unsigned long long off = 0;
            for (uint32_t g = 0; g < world; g++) {
                counts[g] = h[16 + g];
                h[16 + kMaxWorld + g] = off;
                off += h[16 + g];
            }
            PHIP(hipMemcpyAsync(d_cursor, h + 16 + kMaxWorld, world * sizeof(unsigned long long),
                                hipMemcpyHostToDevice, stream));
            timed(KETOGPU_PART_K_PACK, 32 * n,
                  [&] { KLAUNCH(part_scatter_kernel, dim3(grid), dim3(kPB), 0, stream, P, P.obuf, n, d_cursor, send); });
            PHIP(hipGetLastError());
        } else {
            for (uint32_t g = 0; g < world; g++) counts[g] = 0;
        }
        PHIP(hipMemsetAsync(&P.ctr[3], 0, sizeof(unsigned long long), stream));
        // the exchange reads `send` on another stream (torch's, for RCCL); at world 1 the
        // records go straight back into apply on this stream, in order, without a host wait
        if (world > 1) PHIP(hipStreamSynchronize(stream));
        stats.records_sent += n;
        return KETOGPU_OK;
    }

    // an exchange reads `send` (a communicator at world 1): the records are copied there
    bool exchange_pack = false;
    // world 1: the records of the last emit, left in obuf (pack); applying the caller's
    // `send` buffer then means applying obuf.  obuf is rewritten only by the next seed /
    // expand / pull_emit, all after this apply on the same stream.
    const ketogpu_record *obuf_send = nullptr;
    uint64_t obuf_n = 0;
    const ketogpu_record *incoming(const ketogpu_record *recv, uint64_t n) {
        const ketogpu_record *r = (world == 1 && recv && recv == obuf_send && n == obuf_n) ? P.obuf : recv;
        obuf_send = nullptr;
        return r;
    }

    int apply(const ketogpu_record *recv, uint64_t n, uint64_t *frontier) {
        recv = incoming(recv, n);
        const int nxt = cur ^ 1;
        PHIP(hipMemsetAsync(&P.ctr[nxt], 0, sizeof(unsigned long long), stream));
        const uint64_t base = lb + cnt;
        if (n)
            timed(KETOGPU_PART_K_APPLY, 32 * n, [&] {
                KLAUNCH(part_apply_kernel, dim3((unsigned)std::min<uint64_t>((n + kATile - 1) / kATile, 8192)),
                        dim3(kPB), 0, stream, P, recv, n, base, &P.ctr[nxt]);
            });
        read_ctr();
        stats.records_received += n;
        if (overflow_bits()) {
            *frontier = 0;
            return overflow_bits() & 2u ? KETOGPU_EINVAL : KETOGPU_ENOMEM;
        }
        const uint64_t ncnt = h[nxt] >> kCntShift, nedges = h[nxt] & kPreMask;
        stats.bytes[KETOGPU_PART_K_APPLY] += 16 * ncnt;  // appended (key, prefix) entries
        if (ncnt)
            timed(KETOGPU_PART_K_GATHER, 32 * ncnt, [&] {
                KLAUNCH(part_gather_kernel, dim3(pblocks(ncnt)), dim3(kPB), 0, stream, P, base, base + ncnt);
            });
        lb = base;
        cnt = ncnt;
        edges = nedges;
        cur = nxt;
        *frontier = ncnt;
        stats.levels++;
        stats.frontier_entries += ncnt;
        // no host wait for the gather: expand and the next emit's counter read follow it on
        // this stream (each host synchronization left the GPU idle ~20 us per level)
        return KETOGPU_OK;
    }

    void expand() {
        if (cnt && edges) {
            uint64_t tiles = (edges + kPTile - 1) / kPTile;
            unsigned grid = (unsigned)std::min<uint64_t>(tiles, 256ull * 16);
            timed(KETOGPU_PART_K_EXPAND, 40 * cnt + 20 * edges,
                  [&] { KLAUNCH(part_expand_kernel, dim3(grid), dim3(kPB), 0, stream, P, lb, cnt, edges); });
            PHIP(hipGetLastError());
            stats.forward_edges += edges;
        }
        // no host wait: the next emit reads the record counter on this stream first
    }

    void pull_emit() {
        timed(KETOGPU_PART_K_PULL_EMIT, 16 * P.n,
              [&] { KLAUNCH(part_pull_emit_kernel, dim3(pblocks(P.n)), dim3(kPB), 0, stream, P); });
        PHIP(hipGetLastError());
    }

    int pull_answer(const ketogpu_record *recv, uint64_t n) {
        recv = incoming(recv, n);
        if (n)
            timed(KETOGPU_PART_K_PULL_ANSWER, 24 * n,
                  [&] { KLAUNCH(part_pull_answer_kernel, dim3(pblocks(n)), dim3(kPB), 0, stream, P, recv, n); });
        read_ctr();
        stats.queries_answered += n;
        return overflow_bits() & 2u ? KETOGPU_EINVAL : KETOGPU_OK;
    }

    // Clear the round's state.  dense (or after an overflow, when bits may be unrecorded):
    // the whole current buffer, synchronously.  Sparse: the recorded entries, on rstream
    // after the round's last kernel, while the next round runs on the other buffer.
    void reset(bool dense) {
        read_ctr();
        if (dense || overflow_bits()) {
            wait_clean();
            const size_t state = (size_t)W * std::max<uint32_t>(P.Nil, 1);
            PHIP(hipMemsetAsync(P.vis, 0, state * 8, stream));
            PHIP(hipMemsetAsync(P.nxt, 0, state * 8, stream));
        } else {
            const uint64_t ents = lb + cnt, ntouch = h[2];
            PHIP(hipEventRecord(done_ev, stream));
            PHIP(hipStreamWaitEvent(rstream, done_ev, 0));
            uint64_t *vis = P.vis, *keys = P.fe_key, *touch = P.touch;
            const uint32_t Nil = P.Nil;
            if (ents)
                timed(
                    KETOGPU_PART_K_RESET, 16 * ents,
                    [&] { KLAUNCH(part_reset_kernel, dim3(pblocks(ents)), dim3(kPB), 0, rstream, vis, Nil, keys, ents); },
                    rstream);
            if (ntouch)
                timed(
                    KETOGPU_PART_K_RESET, 16 * ntouch,
                    [&] { KLAUNCH(part_reset_kernel, dim3(pblocks(ntouch)), dim3(kPB), 0, rstream, vis, Nil, touch, ntouch); },
                    rstream);
            PHIP(hipEventRecord(clean_ev[vb], rstream));
            clean_pending[vb] = true;
            use_buffer(vb ^ 1);  // the next round's state
        }
        PHIP(hipMemsetAsync(P.ctr, 0, 8 * sizeof(unsigned long long), stream));
        PHIP(hipStreamSynchronize(stream));
        if (timing) resolve_timing();
        lb = cnt = edges = 0;
        dirty = false;
    }

    void end(uint64_t *bits) {
        const uint64_t words = (P.n + 63) / 64;
        if (words && bits) PHIP(hipMemcpyAsync(bits, P.allowed, words * 8, hipMemcpyDeviceToHost, stream));
        PHIP(hipStreamSynchronize(stream));
        reset(false);
    }
};

// ------------------------------------------------- steps of the native round driver
// (part_round.cpp): the C entry points below, so every step keeps its lock and its error
// reporting
namespace ketogpu {
namespace {
struct DeviceSteps : Steps {
    ketogpu_part *p;
    explicit DeviceSteps(ketogpu_part *q) : p(q) {
        device = true;
        dev = q->device;
        stream = q->stream;
    }
    uint64_t round_words() override { return p->W; }
    uint64_t record_capacity() override { return p->P.ocap; }
    int begin(const uint32_t *r, const uint32_t *t, uint64_t n, int dir) override {
        return ketogpu_part_begin_dir(p, r, t, n, dir);
    }
    int emit(int pull, ketogpu_record *send, uint64_t cap, uint64_t *counts) override {
        return pull ? ketogpu_part_pull_emit(p, send, cap, counts) : ketogpu_part_emit(p, send, cap, counts);
    }
    int apply(const ketogpu_record *recv, uint64_t n, uint64_t *frontier) override {
        return ketogpu_part_apply(p, recv, n, frontier);
    }
    int expand() override { return ketogpu_part_expand(p); }
    int pull_answer(const ketogpu_record *recv, uint64_t n) override { return ketogpu_part_pull_answer(p, recv, n); }
    int end(uint64_t *bits) override { return ketogpu_part_end(p, bits); }
    int abort() override { return ketogpu_part_abort(p); }
    void sync() override { (void)ketogpu_part_sync(p); }
    void set_exchange(bool on) override {
        std::lock_guard<std::mutex> lk(p->mu);
        p->exchange_pack = on;
    }
    std::string error() override {
        const char *e = ketogpu_last_error();
        return e ? e : "";
    }
};
}  // namespace
std::unique_ptr<Steps> device_steps(ketogpu_part *p) { return std::make_unique<DeviceSteps>(p); }
}  // namespace ketogpu

// ------------------------------------------------------------------- C ABI
#define PAPI_BEGIN try {
#define PAPI_END                                                                                       \
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

uint32_t ketogpu_part_owner(const ketogpu_part *p, uint32_t node) {
    return p ? part_owner(node, p->P.Ni, p->P.Nx, p->P.world) : 0;
}

int ketogpu_part_new(const ketogpu_shard *s, const ketogpu_part_opts *opts, ketogpu_part **out) {
    PAPI_BEGIN
    if (!s || !opts || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto p = std::make_unique<ketogpu_part>();
    p->init(s, *opts);
    *out = p.release();
    PAPI_END
}

void ketogpu_part_free(ketogpu_part *p) { delete p; }

uint64_t ketogpu_part_round_words(const ketogpu_part *p) { return p ? p->W : 0; }

int ketogpu_part_begin(ketogpu_part *p, const uint32_t *roots, const uint32_t *targets, size_t n) {
    PAPI_BEGIN
    if (!p || (n && (!roots || !targets))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->begin(roots, targets, n, KETOGPU_PART_FORWARD);
    PAPI_END
}

int ketogpu_part_begin_dir(ketogpu_part *p, const uint32_t *roots, const uint32_t *targets, size_t n,
                           int32_t direction) {
    PAPI_BEGIN
    if (!p || (n && (!roots || !targets))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->begin(roots, targets, n, direction);
    PAPI_END
}

int ketogpu_part_emit(ketogpu_part *p, ketogpu_record *send, uint64_t capacity, uint64_t *counts) {
    PAPI_BEGIN
    if (!p || !counts || (capacity && !send)) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    int rc = p->pack(send, capacity, counts);
    if (rc) {
        set_last_error(rc == KETOGPU_EINVAL
                           ? "partition: a request has a node id outside the snapshot"
                           : "partition: outgoing records exceed the buffers; retry with fewer words per round");
        return rc;
    }
    PAPI_END
}

int ketogpu_part_apply(ketogpu_part *p, const ketogpu_record *recv, uint64_t n, uint64_t *frontier) {
    PAPI_BEGIN
    if (!p || !frontier || (n && !recv)) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    int rc = p->apply(recv, n, frontier);
    if (rc) {
        set_last_error(rc == KETOGPU_EINVAL ? "partition: received a record for a node this rank does not own"
                                            : "partition: frontier lists overflow; retry with fewer words per round");
        return rc;
    }
    PAPI_END
}

int ketogpu_part_expand(ketogpu_part *p) {
    PAPI_BEGIN
    if (!p) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->expand();
    PAPI_END
}

int ketogpu_part_pull_emit(ketogpu_part *p, ketogpu_record *send, uint64_t capacity, uint64_t *counts) {
    PAPI_BEGIN
    if (!p || !counts || (capacity && !send)) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->pull_emit();
    int rc = p->pack(send, capacity, counts);
    if (rc) {
        set_last_error("partition: pull queries exceed the buffers; retry with fewer words per round");
        return rc;
    }
    PAPI_END
}

int ketogpu_part_pull_answer(ketogpu_part *p, const ketogpu_record *recv, uint64_t n) {
    PAPI_BEGIN
    if (!p || (n && !recv)) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    if (p->pull_answer(recv, n)) throw Error(KETOGPU_EINVAL, "partition: query for a node this rank does not own");
    PAPI_END
}

int ketogpu_part_end(ketogpu_part *p, uint64_t *allowed_bits) {
    PAPI_BEGIN
    if (!p) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->end(allowed_bits);
    PAPI_END
}

int ketogpu_part_abort(ketogpu_part *p) {
    PAPI_BEGIN
    if (!p) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    p->reset(true);
    PAPI_END
}

int ketogpu_part_sync(ketogpu_part *p) {
    PAPI_BEGIN
    if (!p) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    PHIP(hipStreamSynchronize(p->stream));
    PAPI_END
}

int ketogpu_part_set_timing(ketogpu_part *p, int32_t on) {
    PAPI_BEGIN
    if (!p) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(p->mu);
    PHIP(hipSetDevice(p->device));
    PHIP(hipStreamSynchronize(p->stream));
    if (p->timing) p->resolve_timing();
    p->timing = on != 0;
    PAPI_END
}

int ketogpu_part_stats_get(const ketogpu_part *p, ketogpu_part_stats *out) {
    if (!p || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    *out = p->stats;
    return KETOGPU_OK;
}

}  // extern "C"
