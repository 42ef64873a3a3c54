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
#include <mutex>
#include <string>
#include <vector>

#include "ketogpu_internal.hpp"

using namespace ketogpu;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;
constexpr int kCntShift = 36;  // packed append counter: count << 36 | prefix
constexpr uint64_t kPreMask = (1ull << kCntShift) - 1;
constexpr uint32_t kDynBase = 0x80000000u;

struct DevGraph {
    const uint64_t *fint_off;
    const uint32_t *fint_col;
    const uint64_t *rev_off;
    const uint32_t *rev_col;
    const uint32_t *row_amb;  // nullptr when the snapshot has no ambiguous keys
    uint32_t Ni, Nx, N;
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
};

__device__ __forceinline__ bool bit_of(const uint32_t *bm, uint32_t i) { return (bm[i >> 5] >> (i & 31)) & 1u; }

// 64-lane inclusive scan of a uint64 value
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Append (key, row length) to a frontier list with one atomic per wave.  Every lane of
// the wave must call this (inactive lanes pass want = false).
__device__ __forceinline__ void wave_append(bool want, uint64_t key, uint64_t deg, int lane,
                                            unsigned long long *ctr, uint64_t base, uint64_t cap,
                                            uint64_t *out_key, uint64_t *out_pre, uint64_t *out_mask,
                                            uint64_t mask, unsigned int *overflow) {
    uint64_t val = want ? ((1ull << kCntShift) | deg) : 0ull;
    uint64_t incl = wave_incl_scan(val, lane);
    uint64_t total = __shfl(incl, 63, 64);
    if (!total) return;
    unsigned long long start = 0;
    if (lane == 63) start = atomicAdd(ctr, (unsigned long long)total);
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

// first index in a[0, n) with a[i] > key, computed by one full wave (64-ary search)
__device__ uint64_t wave_upper_bound(const uint64_t *a, uint64_t n, uint64_t key, int lane) {
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
            for (uint64_t p = g.rev_off[t], pe = g.rev_off[t + 1]; p < pe && !ok; p++) {
                uint32_t v = g.rev_col[p];
                examined++;
                if (v == r || (v < g.Ni && ((vrow[v] >> b) & 1ull))) ok = true;
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

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

#define HIP_CHECK(x)                                                                                   \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess)                                                                          \
            throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e));              \
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

// --------------------------------------------------------------------- engine
struct ketogpu_queries {
    uint64_t n = 0;
    uint32_t *d_roots = nullptr, *d_targets = nullptr;
    uint64_t *d_allowed = nullptr, *d_flags = nullptr;
    // dynamic roots of this batch
    uint64_t *d_dyn_int_off = nullptr, *d_dyn_full_off = nullptr;
    uint32_t *d_dyn_int = nullptr, *d_dyn_full = nullptr, *d_dyn_amb = nullptr;
    bool has_dyn = false;
    ~ketogpu_queries() {
        for (void *p : {(void *)d_roots, (void *)d_targets, (void *)d_allowed, (void *)d_flags, (void *)d_dyn_int_off,
                        (void *)d_dyn_full_off, (void *)d_dyn_int, (void *)d_dyn_full, (void *)d_dyn_amb})
            if (p) (void)hipFree(p);
    }
};

struct ketogpu_engine {
    const Snapshot *snap = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevGraph g{};
    DevState st{};
    uint64_t Wmax = 0;
    uint64_t *h_ctr = nullptr;  // pinned
    std::vector<void *> owned;
    ketogpu_run_stats last{};
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;

    hipEvent_t ev() {
        if (ev_used == ev_pool.size()) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            ev_pool.push_back(e);
        }
        return ev_pool[ev_used++];
    }

    ~ketogpu_engine() {
        if (stream) {
            (void)hipSetDevice(device);
            (void)hipStreamSynchronize(stream);
        }
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        for (void *p : owned) (void)hipFree(p);
        if (h_ctr) (void)hipHostFree(h_ctr);
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
        if (s.N >= kDynBase) throw Error(KETOGPU_EINVAL, "snapshot has >= 2^31 nodes");
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

        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        uint64_t budget = o && o->state_budget_bytes ? o->state_budget_bytes
                                                     : std::min<uint64_t>(free_b / 4, (uint64_t)64 << 30);
        budget = std::min<uint64_t>(budget, (uint64_t)free_b * 3 / 4);
        // frontier lists: 24 B per entry, touch list 8 B; vis+nxt: 16 B per (word, node)
        uint64_t lists = std::min<uint64_t>(budget / 4, (uint64_t)24 << 30);
        st.fe_cap = std::max<uint64_t>(lists / 32, 1 << 16);
        st.touch_cap = st.fe_cap;
        uint64_t per_word = 16ull * std::max<uint32_t>(s.Ni, 1);
        Wmax = std::max<uint64_t>(1, (budget - std::min(budget, lists)) / per_word);
        if (o && o->max_words_per_round) Wmax = std::min<uint64_t>(Wmax, o->max_words_per_round);
        Wmax = std::min<uint64_t>(Wmax, 1u << 20);
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
        st.stats = dalloc<unsigned long long>(8);
        for (void *p : {(void *)st.ctr, (void *)st.overflow, (void *)st.stats}) owned.push_back(p);
        HIP_CHECK(hipHostMalloc((void **)&h_ctr, 16 * sizeof(uint64_t), hipHostMallocDefault));
        HIP_CHECK(hipStreamSynchronize(stream));
    }

    // read ctr[0..2] and overflow into h_ctr[0..3]
    void read_counters() {
        HIP_CHECK(hipMemcpyAsync(h_ctr, st.ctr, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipMemcpyAsync(h_ctr + 3, st.overflow, sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
    }

    // One round over requests [c0, c0 + n) (c0 multiple of 64).  Returns false on list
    // overflow (state is then dense-reset and the caller splits the round).
    bool round(ketogpu_queries &q, uint64_t c0, uint64_t n, ketogpu_run_stats &rs,
               std::vector<std::pair<hipEvent_t, hipEvent_t>> &push_ev,
               std::vector<std::pair<hipEvent_t, hipEvent_t>> &pull_ev) {
        const uint64_t W = (n + 63) / 64;
        const uint64_t wg0 = c0 / 64;
        HIP_CHECK(hipMemsetAsync(st.ctr, 0, 3 * sizeof(uint64_t), stream));
        HIP_CHECK(hipMemsetAsync(st.overflow, 0, sizeof(unsigned int), stream));
        *(uint64_t *)&h_ctr[3] = 0;
        hipLaunchKernelGGL(seed_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.d_roots, q.d_targets,
                           c0, n, q.d_flags);
        read_counters();
        uint64_t cnt = h_ctr[0] >> kCntShift, edges = h_ctr[0] & kPreMask;
        std::vector<uint64_t> level_begin{0};
        uint64_t lb = 0;
        int cur = 0;  // ctr index of the current level
        if (q.has_dyn) {
            hipLaunchKernelGGL(seed_dynamic_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.d_roots,
                               q.d_targets, c0, n, q.d_dyn_int_off, q.d_dyn_int, q.d_dyn_amb, q.d_flags, lb + cnt,
                               &st.ctr[1]);
        }
        bool overflow = (uint32_t)h_ctr[3] != 0;
        for (uint64_t level = 0; !overflow; level++) {
            if (level > 0 && cnt)
                hipLaunchKernelGGL(gather_kernel, dim3(blocks_for(cnt)), dim3(kBlock), 0, stream, g, st, lb, lb + cnt);
            bool dyn_pending = level == 0 && q.has_dyn;
            if (!cnt && !dyn_pending) break;
            int nxt = cur ^ 1;
            if (level > 0) HIP_CHECK(hipMemsetAsync(&st.ctr[nxt], 0, sizeof(uint64_t), stream));
            if (edges) {
                uint64_t tiles = (edges + kTile - 1) / kTile;
                unsigned grid = (unsigned)std::min<uint64_t>(tiles, 256ull * 16);
                hipEvent_t a = ev(), b = ev();
                HIP_CHECK(hipEventRecord(a, stream));
                hipLaunchKernelGGL(expand_kernel, dim3(grid), dim3(kBlock), 0, stream, g, st, lb, cnt, edges, lb + cnt,
                                   &st.ctr[nxt], q.d_flags, wg0);
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
            HIP_CHECK(hipMemsetAsync(q.d_flags + wg0, 0, W * 8, stream));
            HIP_CHECK(hipStreamSynchronize(stream));
            return false;
        }
        // pull: one thread per request
        hipEvent_t a = ev(), b = ev();
        HIP_CHECK(hipEventRecord(a, stream));
        hipLaunchKernelGGL(pull_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, stream, g, st, q.d_roots, q.d_targets, c0, n,
                           q.d_dyn_full_off, q.d_dyn_full, q.d_allowed);
        HIP_CHECK(hipEventRecord(b, stream));
        pull_ev.push_back({a, b});
        // reset every visited entry recorded in this round (levels >= 1 and touch list)
        uint64_t first = level_begin.size() > 1 ? level_begin[1] : lb;
        if (lb > first)
            hipLaunchKernelGGL(reset_kernel, dim3(blocks_for(lb - first)), dim3(kBlock), 0, stream, st.vis, g.Ni,
                               st.fe_key + first, lb - first);
        uint64_t ntouch = h_ctr[2];
        if (ntouch)
            hipLaunchKernelGGL(reset_kernel, dim3(blocks_for(ntouch)), dim3(kBlock), 0, stream, st.vis, g.Ni, st.touch,
                               ntouch);
        rs.touched += (lb - first) + ntouch;
        rs.rounds++;
        return true;
    }

    void run(ketogpu_queries &q) {
        HIP_CHECK(hipSetDevice(device));
        ketogpu_run_stats rs{};
        rs.checks = q.n;
        ev_used = 0;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> push_ev, pull_ev;
        hipEvent_t t_begin = ev(), t_end = ev();
        uint64_t words = (q.n + 63) / 64;
        HIP_CHECK(hipMemsetAsync(st.stats, 0, 8 * sizeof(uint64_t), stream));
        HIP_CHECK(hipMemsetAsync(q.d_flags, 0, std::max<uint64_t>(words, 1) * 8, stream));
        HIP_CHECK(hipEventRecord(t_begin, stream));
        uint64_t W = Wmax;
        for (uint64_t w0 = 0; w0 < words;) {
            uint64_t wn = std::min<uint64_t>(W, words - w0);
            uint64_t c0 = w0 * 64, n = std::min<uint64_t>(q.n - c0, wn * 64);
            if (!round(q, c0, n, rs, push_ev, pull_ev)) {
                rs.overflow_retries++;
                if (wn == 1) throw Error(KETOGPU_ENOMEM, "frontier list overflow for a single 64-request word");
                W = std::max<uint64_t>(1, wn / 2);
                continue;
            }
            w0 += wn;
        }
        HIP_CHECK(hipEventRecord(t_end, stream));
        uint64_t examined = 0;
        HIP_CHECK(hipMemcpyAsync(h_ctr + 8, st.stats, sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
        examined = h_ctr[8];
        rs.rev_edges = examined;
        // pull bytes: 16 per request row open (rev_off), 4 per reverse entry, 8 per
        // visited-word read, 8 per result word
        rs.bytes_pull = 16 * q.n + 4 * examined + 8 * examined + 8 * words;
        rs.bytes_total = rs.bytes_push + rs.bytes_pull + 8 * 2 * rs.touched;
        float ms = 0;
        for (auto &p : push_ev) {
            HIP_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
            rs.ms_push += ms;
        }
        for (auto &p : pull_ev) {
            HIP_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
            rs.ms_pull += ms;
        }
        HIP_CHECK(hipEventElapsedTime(&ms, t_begin, t_end));
        rs.ms_total = ms;
        last = rs;
    }

    ketogpu_queries *upload(const uint32_t *roots, const uint32_t *targets, uint64_t n) {
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
        HIP_CHECK(hipStreamSynchronize(stream));
        return q.release();
    }

    void download(const ketogpu_queries &q, uint64_t *allowed, uint64_t *flagged) {
        HIP_CHECK(hipSetDevice(device));
        uint64_t words = (q.n + 63) / 64;
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
    e->init(*reinterpret_cast<const Snapshot *>(s), opts);
    *out = e.release();
    API_END
}

void ketogpu_engine_free(ketogpu_engine *e) { delete e; }

int ketogpu_queries_upload(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                           ketogpu_queries **out) {
    API_BEGIN
    if (!e || !out || (n && (!roots || !targets))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    const Snapshot &s = *e->snap;
    for (size_t i = 0; i < n; i++)  // never launch on ids the graph does not have
        if ((roots[i] != NONE && roots[i] >= s.Nx) || (targets[i] != NONE && targets[i] >= s.N))
            throw Error(KETOGPU_EINVAL, "request " + std::to_string(i) + " has a node id outside the snapshot");
    *out = e->upload(roots, targets, n);
    API_END
}

int ketogpu_queries_run(ketogpu_engine *e, ketogpu_queries *q) {
    API_BEGIN
    if (!e || !q) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    e->run(*q);
    API_END
}

int ketogpu_queries_download(ketogpu_engine *e, const ketogpu_queries *q, uint64_t *allowed_bits,
                             uint64_t *flagged_bits) {
    API_BEGIN
    if (!e || !q) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    e->download(*q, allowed_bits, flagged_bits);
    API_END
}

void ketogpu_queries_free(ketogpu_queries *q) { delete q; }

int ketogpu_check_ids(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                      uint64_t *allowed_bits, uint64_t *flagged_bits) {
    ketogpu_queries *q = nullptr;
    int rc = ketogpu_queries_upload(e, roots, targets, n, &q);
    if (rc) return rc;
    std::unique_ptr<ketogpu_queries> owned(q);
    if ((rc = ketogpu_queries_run(e, q))) return rc;
    return ketogpu_queries_download(e, q, allowed_bits, flagged_bits);
}

int ketogpu_check(ketogpu_engine *e, const ketogpu_check_request *reqs, size_t n, uint8_t *allowed, int32_t *status) {
    API_BEGIN
    if (!e || (n && (!reqs || !allowed))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
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
    std::unique_ptr<ketogpu_queries> q(e->upload(roots.data(), targets.data(), n));
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

int ketogpu_engine_last_stats(const ketogpu_engine *e, ketogpu_run_stats *out) {
    if (!e || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    *out = e->last;
    return KETOGPU_OK;
}

}  // extern "C"
