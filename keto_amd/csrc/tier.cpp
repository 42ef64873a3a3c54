// tier.cpp — the two-tier partitioned mode: host state and exchange protocol
// (include/ketogpu.h "two-tier"; kernels in device_engine.hip, shared declarations in
// tier.hpp).
//
// Why two tiers.  The per-level partitioned engine (partition.hip, part_round.cpp) moves a
// frontier record for every (request, node) a BFS level reaches — 359 records per check
// on config #5's shape — through two collectives per level, and keeps 64-request state
// words in HBM for every owned interior node.  But in Keto's data model every check path
// r -> v1 -> ... -> v(k-1) -> t (internal/check/engine.go:33-91: subjectIsAllowed
// recursing through checkOneIndirectionFurther) starts with a row of r's and ends with a
// row containing t; only its middle runs among interior nodes (subject sets that appear
// as subjects).  Those rows — the core — are group nesting, a small part of an RBAC or
// social network (config #5: ~0.3% of the tuples), so every rank keeps a copy and the
// only rows that travel are the two seed rows of each request:
//
//   [agree on the number of steps: every rank's batch size]
//   per step:  queries -> [all-gather counts + status] -> [all-to-all]
//           -> replies -> [all-gather counts + status] -> [all-to-all]
//           -> evaluate (lite_unit on the local core; the cascade of larger tables)
//           -> [all-gather status + unfinished requests] -> per-level engine for those
//
// One rank (no communicator) needs no exchange: its own rows are read in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "core_index.hpp"  // parallel_chunks
#include "labels.hpp"
#include "part_round.hpp"
#include "tier.hpp"

using namespace ketogpu;

namespace {

#define THIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// kernels' statistics buffer: 8 words + 1024 slots of 4 (device_engine.hip kStatsLen)
constexpr size_t kEvalStatsLen = 8 + 8 * 1024 + 8 + 4;

// ---------------------------------------------------------------- buffers
// a growable buffer in device memory (of `dev`) or host memory
struct Buf {
    void *p = nullptr;
    uint64_t cap = 0;
    bool device = false;
    int dev = -1;
    Buf() = default;
    Buf(const Buf &) = delete;
    ~Buf() { release(); }
    void release() {
        if (!p) return;
        if (device)
            (void)hipFree(p);
        else
            free(p);
        p = nullptr;
        cap = 0;
    }
    void *ensure(uint64_t bytes) {
        bytes = std::max<uint64_t>(bytes, 256);
        if (bytes <= cap) return p;
        release();
        const uint64_t want = bytes + bytes / 2;
        if (device) {
            THIP(hipSetDevice(dev));
            if (hipMalloc(&p, want) != hipSuccess) {
                (void)hipGetLastError();
                p = nullptr;
                throw Error(KETOGPU_ENOMEM, "two-tier: out of device memory for exchange buffers");
            }
        } else {
            p = malloc(want);
            if (!p) throw std::bad_alloc();
        }
        cap = want;
        return p;
    }
    template <class T>
    T *as() const {
        return (T *)p;
    }
};

}  // namespace

// -------------------------------------------------------------------- core
struct ketogpu_core {
    uint64_t Ni = 0;
    std::vector<uint64_t> f_off, b_off;
    std::vector<uint32_t> f_col, b_col;
    uint64_t bytes() const { return 16 * (f_col.size() + b_col.size()); }
};

namespace {

// Every rank's owned interior rows (forward: interior successors; backward: interior
// predecessors) gathered into the core on every rank.  Payload of a rank: nil, then per
// owned interior local its two row lengths, then the rows.
std::unique_ptr<ketogpu_core> gather_core(const ketogpu_shard_graph &v, Comm *comm, uint64_t budget) {
    const uint64_t nil = v.owned_interior;
    std::vector<uint32_t> mine;
    mine.reserve(1 + 2 * nil + v.lf_off[nil] + v.lb_off[nil]);
    mine.push_back((uint32_t)nil);
    for (uint64_t l = 0; l < nil; l++) {
        mine.push_back((uint32_t)(v.lf_off[l + 1] - v.lf_off[l]));
        mine.push_back((uint32_t)(v.lb_off[l + 1] - v.lb_off[l]));
    }
    mine.insert(mine.end(), v.lf_col, v.lf_col + v.lf_off[nil]);
    mine.insert(mine.end(), v.lb_col, v.lb_col + v.lb_off[nil]);
    const uint32_t W = v.world;
    std::vector<std::vector<uint32_t>> parts(W);
    if (!comm || W == 1) {
        parts[0] = std::move(mine);
    } else {
        HostColl hc(comm);
        // the budget is agreed before anything large moves: every rank's core bytes
        uint64_t ef = v.lf_off[nil], eb = v.lb_off[nil];
        const auto &m = hc.gather({ef, eb});
        uint64_t tf = 0, tb = 0;
        for (uint32_t r = 0; r < W; r++) tf += m[2 * r], tb += m[2 * r + 1];
        if (budget && 16 * (tf + tb) > budget)
            throw Error(KETOGPU_ENOMEM, "two-tier: the core needs " + std::to_string(16 * (tf + tb)) +
                                            " bytes of records, over the budget of " + std::to_string(budget));
        std::vector<uint64_t> sizes;
        std::vector<char> all = hc.allgatherv(mine.data(), mine.size() * 4, &sizes);
        uint64_t at = 0;
        for (uint32_t r = 0; r < W; r++) {
            parts[r].resize(sizes[r] / 4);
            if (sizes[r]) memcpy(parts[r].data(), all.data() + at, sizes[r]);
            at += sizes[r];
        }
    }
    auto c = std::make_unique<ketogpu_core>();
    const uint64_t Ni = v.num_interior;
    c->Ni = Ni;
    std::vector<uint64_t> fl(Ni + 1, 0), bl(Ni + 1, 0);
    for (uint32_t r = 0; r < W; r++) {
        const auto &p = parts[r];
        if (p.empty()) throw Error(KETOGPU_EINVAL, "two-tier: a rank sent no core rows");
        const uint64_t n = p[0];
        for (uint64_t l = 0; l < n; l++) {
            const uint64_t g = l * W + r;
            if (g >= Ni) throw Error(KETOGPU_EINVAL, "two-tier: a core row outside the interior range");
            fl[g + 1] = p[1 + 2 * l];
            bl[g + 1] = p[2 + 2 * l];
        }
    }
    for (uint64_t g = 0; g < Ni; g++) fl[g + 1] += fl[g], bl[g + 1] += bl[g];
    if (budget && 16 * (fl[Ni] + bl[Ni]) > budget)
        throw Error(KETOGPU_ENOMEM, "two-tier: the core needs " + std::to_string(16 * (fl[Ni] + bl[Ni])) +
                                        " bytes of records, over the budget of " + std::to_string(budget));
    if (fl[Ni] >= (1ull << 32) || bl[Ni] >= (1ull << 32))
        throw Error(KETOGPU_ENOMEM, "two-tier: the core has 2^32 or more rows entries (32-bit record begins)");
    c->f_off = fl;
    c->b_off = bl;
    c->f_col.resize(fl[Ni]);
    c->b_col.resize(bl[Ni]);
    for (uint32_t r = 0; r < W; r++) {
        const auto &p = parts[r];
        const uint64_t n = p[0];
        uint64_t at = 1 + 2 * n;
        for (uint64_t l = 0; l < n; l++) {  // forward rows first, then backward rows
            const uint64_t g = l * W + r, len = p[1 + 2 * l];
            if (at + len > p.size()) throw Error(KETOGPU_EINVAL, "two-tier: a truncated core payload");
            std::copy(p.begin() + at, p.begin() + at + len, c->f_col.begin() + fl[g]);
            at += len;
        }
        for (uint64_t l = 0; l < n; l++) {
            const uint64_t g = l * W + r, len = p[2 + 2 * l];
            if (at + len > p.size()) throw Error(KETOGPU_EINVAL, "two-tier: a truncated core payload");
            std::copy(p.begin() + at, p.begin() + at + len, c->b_col.begin() + bl[g]);
            at += len;
        }
    }
    for (uint32_t x : c->f_col)
        if (x >= Ni) throw Error(KETOGPU_EINVAL, "two-tier: a core row entry outside the interior");
    for (uint32_t x : c->b_col)
        if (x >= Ni) throw Error(KETOGPU_EINVAL, "two-tier: a core row entry outside the interior");
    return c;
}

bool device_memory(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice;
}

// --------------------------------------------------------------- steps
// One rank's steps of a two-tier batch (device: TierDevice below; tests: the caller's
// vtable over host memory).  Codes are KETOGPU_*.
struct TierSteps {
    bool device = false;
    int dev = -1;
    hipStream_t stream = nullptr;
    virtual ~TierSteps() = default;
    virtual int queries(const uint32_t *roots, const uint32_t *targets, uint64_t n, tier::Query *send,
                        uint64_t *counts) = 0;
    virtual int reply_sizes(const tier::Query *recv, uint64_t n, const uint64_t *from, uint64_t *counts) = 0;
    virtual int reply_emit(tier::Reply *send, uint64_t cap) = 0;
    // recv null: the rank owns every root and target (world 1)
    virtual int evaluate(const uint32_t *roots, const uint32_t *targets, uint64_t n, const tier::Reply *recv,
                         uint64_t nrecv, uint64_t *bits, std::vector<uint32_t> &overflow) = 0;
    virtual void stats(ketogpu_tier_stats &) {}
    virtual std::string error() = 0;
    // bytes per reply item (tier::Reply; plan label: 4-byte words, tier.hpp "label replies")
    virtual uint64_t reply_unit() const { return sizeof(tier::Reply); }
    // the reply items received from each source this step (before evaluate)
    virtual void replies_from(const uint64_t *, int) {}
    // world 1 with one host wait (TierDevice::step_world1), when the steps have it
    virtual bool has_world1() const { return false; }
    virtual int step_world1(const uint32_t *, const uint32_t *, uint64_t, uint64_t *, std::vector<uint32_t> &,
                            uint64_t &) {
        return KETOGPU_EINVAL;
    }
};

struct VtableTier : TierSteps {
    ketogpu_tier_steps v{};
    std::string err;
    int rc(int code, const char *what) {
        if (code) err = std::string("two-tier steps: ") + what + " returned " + std::to_string(code);
        return code;
    }
    int queries(const uint32_t *r, const uint32_t *t, uint64_t n, tier::Query *send, uint64_t *counts) override {
        return rc(v.queries(v.ctx, r, t, n, (ketogpu_tier_query *)send, counts), "queries");
    }
    int reply_sizes(const tier::Query *recv, uint64_t n, const uint64_t *from, uint64_t *counts) override {
        return rc(v.reply_sizes(v.ctx, (const ketogpu_tier_query *)recv, n, from, counts), "reply_sizes");
    }
    int reply_emit(tier::Reply *send, uint64_t) override {
        return rc(v.reply_emit(v.ctx, (ketogpu_tier_rec *)send), "reply_emit");
    }
    int evaluate(const uint32_t *r, const uint32_t *t, uint64_t n, const tier::Reply *recv, uint64_t nrecv, uint64_t *bits,
                 std::vector<uint32_t> &overflow) override {
        overflow.assign(std::max<uint64_t>(n, 1), 0);
        uint64_t no = 0;
        const int code = rc(v.evaluate(v.ctx, r, t, n, (const ketogpu_tier_rec *)recv, nrecv, bits, overflow.data(), &no),
                            "evaluate");
        overflow.resize(code ? 0 : std::min<uint64_t>(no, n));
        return code;
    }
    std::string error() override { return err; }
};

// ------------------------------------------------------------ device steps
struct TierDevice : TierSteps {
    tier::Graph G{};
    std::vector<void *> owned;
    int n_cu = 256;
    uint64_t core_records = 0, seed_records = 0;
    // KETOGPU_TEST_TIER_OVERFLOW=1 when the engine is made (tests): every request is reported
    // unfinished, its bit cleared, so the per-level engine answers the whole batch
    bool force_overflow = false;
    std::string err;
    // per-step scratch (grown on demand)
    Buf d_req, d_lens, d_scan, d_bnd, d_seed, d_bits, d_list[3], d_srcb;
    unsigned long long *d_small = nullptr;  // [0..63] counts, [64..127] cursors, [128] first_bad, [129] bad query,
                                            // [130..132] list counts, [136..] stats, [kSeg..] label segments
    uint64_t *h_small = nullptr;            // pinned mirror
    uint64_t *d_hsmall = nullptr;           // its device view (tier_emit_kernel writes the status words there)
    // the current step's requests (device-readable) and replies in flight
    const uint32_t *cur_r = nullptr, *cur_t = nullptr, *src_r = nullptr, *src_t = nullptr;
    uint64_t cur_n = 0;
    bool in_place = false;  // cur_r / cur_t are the caller's buffers (a pinned view, or HBM)
    bool req_hbm = false;   // ... in this device's memory: read in place by every pass
    const tier::Query *rq = nullptr;
    uint64_t rq_n = 0;
    // the first evaluation stage bracketed by events (the roofline's kernel time)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double eval_ms = 0;
    uint64_t eval_launches = 0;
    // plan label (KETOGPU_TIER_LABEL, default 1): the owned nodes' label lists answer the
    // queries and the evaluation is one intersection per request (labels.hpp)
    uint64_t label_words = 0;
    double label_ms = 0;

    static constexpr size_t kCounts = 0, kCursor = 64, kFirstBad = 128, kBadQuery = 129, kLists = 130, kStats = 136;
    // label replies: segments' first items, 65 words each: received queries (owner side),
    // sent queries and received words (asker side)
    static constexpr size_t kSeg = kStats + kEvalStatsLen, kQs = kSeg, kSq = kSeg + 72, kRp = kSeg + 144;
    static constexpr size_t kSmall = kSeg + 216;
    // the step's sent queries (label replies are matched to them by position)
    const tier::Query *sent = nullptr;
    std::vector<uint64_t> sent_counts, recv_from;

    ~TierDevice() override {
        if (stream) {
            (void)hipSetDevice(dev);
            (void)hipStreamSynchronize(stream);
        }
        for (Buf *b : {&d_req, &d_lens, &d_scan, &d_bnd, &d_seed, &d_bits, &d_list[0], &d_list[1], &d_list[2], &d_q, &d_rep,
                       &d_srcb})
            b->release();
        for (void *p : owned) (void)hipFree(p);
        for (hipEvent_t e : {ev0, ev1})
            if (e) (void)hipEventDestroy(e);
        if (d_small) (void)hipFree(d_small);
        if (h_small) (void)hipHostFree(h_small);
        if (stream) (void)hipStreamDestroy(stream);
    }

    template <class T>
    T *upload(const T *src, size_t n) {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(KETOGPU_ENOMEM, "two-tier: out of device memory for the graph");
        }
        owned.push_back(p);
        if (n) THIP(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
        return (T *)p;
    }

    // records of rows [off[0], off[rows]) of col: entry x -> (x, its core row); x >= Ni:
    // (x, 0, 0) (a backward entry outside the interior).  Built and uploaded in slices.
    tier::Rec *records(const uint64_t *off, size_t rows, const uint32_t *col, const std::vector<uint64_t> &core_off,
                       uint64_t Ni) {
        const uint64_t n = off[rows];
        void *p = nullptr;
        if (hipMalloc(&p, std::max<uint64_t>(n, 1) * sizeof(tier::Rec)) != hipSuccess) {
            (void)hipGetLastError();
            throw Error(KETOGPU_ENOMEM, "two-tier: out of device memory for the graph");
        }
        owned.push_back(p);
        std::vector<tier::Rec> slice;
        const uint64_t step = 1 << 24;
        for (uint64_t b = 0; b < n; b += step) {
            const uint64_t e = std::min(n, b + step);
            slice.resize(e - b);
            for (uint64_t k = b; k < e; k++) {
                const uint32_t x = col[k];
                slice[k - b] = x < Ni ? tier::Rec{x, (uint32_t)(core_off[x + 1] - core_off[x]), (uint32_t)core_off[x], 0}
                                      : tier::Rec{x, 0, 0, 0};
            }
            THIP(hipMemcpy((tier::Rec *)p + b, slice.data(), (e - b) * sizeof(tier::Rec), hipMemcpyHostToDevice));
        }
        return (tier::Rec *)p;
    }

    void init(const ketogpu_shard *sh, const ketogpu_core *core, int device) {
        ketogpu_shard_graph v{};
        if (const int rc = ketogpu_shard_view(sh, &v)) throw Error(rc, ketogpu_last_error());
        ketogpu_shard_stats ss{};
        if (ketogpu_shard_stats_get(sh, &ss) == KETOGPU_OK && ss.ambiguous_keys)
            throw Error(KETOGPU_EINVAL, "two-tier: the graph has ambiguous Subject.String() keys (R4)");
        if (core->Ni != v.num_interior) throw Error(KETOGPU_EINVAL, "two-tier: the core belongs to another layout");
        int ndev = 0;
        THIP(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) throw Error(KETOGPU_EDEVICE, "no such HIP device");
        this->device = true;
        dev = device;
        force_overflow = getenv("KETOGPU_TEST_TIER_OVERFLOW") != nullptr;
        const char *ow = getenv("KETOGPU_TIER_ONE_WAIT");
        one_wait = !ow || atoi(ow) != 0;
        THIP(hipSetDevice(dev));
        THIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        THIP(hipEventCreate(&ev0));
        THIP(hipEventCreate(&ev1));
        THIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
        for (Buf *b : {&d_req, &d_lens, &d_scan, &d_bnd, &d_seed, &d_bits, &d_list[0], &d_list[1], &d_list[2], &d_q, &d_rep,
                       &d_srcb}) {
            b->device = true;
            b->dev = dev;
        }
        THIP(hipMalloc(&d_small, kSmall * 8));
        THIP(hipMemset(d_small, 0, kSmall * 8));
        THIP(hipHostMalloc((void **)&h_small, kSmall * 8, hipHostMallocDefault));
        THIP(hipHostGetDevicePointer((void **)&d_hsmall, h_small, 0));
        G.world = v.world;
        G.rank = v.rank;
        G.Ni = v.num_interior;
        G.Nx = v.num_expandable;
        G.N = v.num_nodes;
        G.Nil = v.owned_interior;
        G.Nxl = v.owned_expandable;
        G.Nl = v.owned_nodes;
        G.both_max = 12;  // device_engine.hip kBothMax / kSeedBothMax: the lite plan's thresholds
        G.seed_max = 32;
        const uint64_t Ni = core->Ni;
        G.core_f = records(core->f_off.data(), Ni, core->f_col.data(), core->f_off, Ni);
        G.core_b = records(core->b_off.data(), Ni, core->b_col.data(), core->b_off, Ni);
        {  // {begin, count} per interior node, one 8-byte read per received entry (u32 like the
           // records' begin fields)
            std::vector<uint2> o(Ni);
            for (uint64_t x = 0; x < Ni; x++)
                o[x] = make_uint2((uint32_t)core->f_off[x], (uint32_t)(core->f_off[x + 1] - core->f_off[x]));
            G.core_f_row = upload(o.data(), o.size());
            for (uint64_t x = 0; x < Ni; x++)
                o[x] = make_uint2((uint32_t)core->b_off[x], (uint32_t)(core->b_off[x + 1] - core->b_off[x]));
            G.core_b_row = upload(o.data(), o.size());
        }
        G.lf_off = upload(v.lf_off, (size_t)v.owned_expandable + 1);
        G.lr_off = upload(v.lr_off, (size_t)v.owned_nodes + 1);
        G.lf_rec = records(v.lf_off, v.owned_expandable, v.lf_col, core->f_off, Ni);
        G.lr_rec = records(v.lr_off, v.owned_nodes, v.lr_col, core->b_off, Ni);
        G.lf_node = upload(v.lf_col, (size_t)v.lf_off[v.owned_expandable]);
        G.lr_node = upload(v.lr_col, (size_t)v.lr_off[v.owned_nodes]);
        G.lf_base = (int64_t)((intptr_t)G.lf_rec - (intptr_t)G.core_f) / (int64_t)sizeof(tier::Rec);
        G.lr_base = (int64_t)((intptr_t)G.lr_rec - (intptr_t)G.core_b) / (int64_t)sizeof(tier::Rec);
        core_records = core->f_col.size() + core->b_col.size();
        seed_records = v.lf_off[v.owned_expandable] + v.lr_off[v.owned_nodes];
        const char *lab = getenv("KETOGPU_TIER_LABEL");
        if (!lab || atoi(lab) != 0) build_label_lists(v, core);
        THIP(hipDeviceSynchronize());
    }

    // The 2-hop labels of the replicated core (the same on every rank: it is the same core)
    // and, per owned node, its S list (labels.hpp: Lin of the interior entries of rev(x) +
    // the other entries) and per owned expandable node its P list (Lout(x) for an interior
    // x, else {x} + Lout of fint(x)), each stored as [mask lo, mask hi, entries ascending].
    void build_label_lists(const ketogpu_shard_graph &v, const ketogpu_core *core) {
        const auto t0 = Clock::now();
        ReachLabels R;
        build_reach_labels_csr((uint32_t)core->Ni, core->f_off.data(), core->f_col.data(), core->b_off.data(),
                               core->b_col.data(), R);
        const uint32_t W = v.world, rank = v.rank;
        const uint64_t Nil = v.owned_interior, Nxl = v.owned_expandable, Nl = v.owned_nodes;
        auto global = [&](uint64_t l) -> uint64_t {
            if (l < Nil) return l * W + rank;
            if (l < Nxl) return v.num_interior + (l - Nil) * W + rank;
            return v.num_expandable + (l - Nxl) * W + rank;
        };
        auto add_out = [&](uint32_t x, std::vector<uint32_t> &o, uint64_t &m) {
            m |= R.mout[x];
            o.insert(o.end(), R.out.begin() + (ptrdiff_t)R.out_off[x], R.out.begin() + (ptrdiff_t)R.out_off[x + 1]);
        };
        // one node's list (p: P side) into o, mask into m
        auto list = [&](bool p, uint64_t l, std::vector<uint32_t> &o, uint64_t &m) {
            o.clear();
            m = 0;
            if (p) {
                const uint64_t g = global(l);
                if (g < R.n) {
                    add_out((uint32_t)g, o, m);
                    return;  // Lout is ascending already
                }
                o.push_back((uint32_t)g);
                for (uint64_t k = v.lf_off[l]; k < v.lf_off[l + 1]; k++) add_out(v.lf_col[k], o, m);
            } else {
                for (uint64_t k = v.lr_off[l]; k < v.lr_off[l + 1]; k++) {
                    const uint32_t x = v.lr_col[k];
                    if (x < R.n) {
                        m |= R.min[x];
                        o.insert(o.end(), R.in.begin() + (ptrdiff_t)R.in_off[x], R.in.begin() + (ptrdiff_t)R.in_off[x + 1]);
                    } else {
                        o.push_back(x);
                    }
                }
            }
            std::sort(o.begin(), o.end());
            o.erase(std::unique(o.begin(), o.end()), o.end());
        };
        auto build = [&](bool p, uint64_t nodes, const uint64_t *&d_off, const uint32_t *&d_col) {
            std::vector<uint64_t> off(nodes + 1, 0);
            parallel_chunks(nodes, 1 << 14, [&](int, uint64_t b, uint64_t e) {
                std::vector<uint32_t> o;
                uint64_t m;
                for (uint64_t l = b; l < e; l++) {
                    list(p, l, o, m);
                    off[l + 1] = 2 + o.size();
                }
            });
            for (uint64_t l = 0; l < nodes; l++) off[l + 1] += off[l];
            std::vector<uint32_t> col(off[nodes]);
            parallel_chunks(nodes, 1 << 14, [&](int, uint64_t b, uint64_t e) {
                std::vector<uint32_t> o;
                uint64_t m;
                for (uint64_t l = b; l < e; l++) {
                    list(p, l, o, m);
                    uint32_t *w = col.data() + off[l];
                    w[0] = (uint32_t)m;
                    w[1] = (uint32_t)(m >> 32);
                    std::copy(o.begin(), o.end(), w + 2);
                }
            });
            label_words += col.size();
            d_off = upload(off.data(), off.size());
            d_col = upload(col.data(), col.size());
        };
        build(false, Nl, G.ls_off, G.ls_col);
        build(true, Nxl, G.lp_off, G.lp_col);
        G.label = 1;
        label_ms = ms_since(t0);
    }

    // the step's requests as the device reads them: pinned memory in place, else copied.
    // fresh = false: the same step's second use (evaluate after queries) keeps the copy.
    void set_requests(const uint32_t *r, const uint32_t *t, uint64_t n, bool fresh) {
        if (!fresh && r == src_r && t == src_t && n == cur_n && cur_r) return;
        src_r = r;
        src_t = t;
        cur_n = n;
        bool dr = false, dt = false;
        cur_r = (const uint32_t *)host_view(r, dev, true, &dr);
        cur_t = cur_r ? (const uint32_t *)host_view(t, dev, true, &dt) : nullptr;
        in_place = cur_r && cur_t;
        req_hbm = in_place && dr && dt;
        if (!in_place) {
            uint32_t *d = (uint32_t *)d_req.ensure(8 * std::max<uint64_t>(n, 1));
            if (n) {
                THIP(hipMemcpyAsync(d, r, 4 * n, hipMemcpyHostToDevice, stream));
                THIP(hipMemcpyAsync(d + n, t, 4 * n, hipMemcpyHostToDevice, stream));
            }
            cur_r = d;
            cur_t = d + n;
        }
    }

    int guarded(const char *what, const std::function<void()> &f) {
        try {
            f();
            return KETOGPU_OK;
        } catch (const Error &e) {
            err = std::string(what) + ": " + e.what();
            return e.code;
        } catch (const std::bad_alloc &) {  // host allocations of a step (lists, overflow)
            err = std::string(what) + ": out of host memory";
            return KETOGPU_ENOMEM;
        } catch (const std::exception &e) {
            err = std::string(what) + ": " + e.what();
            return KETOGPU_EDEVICE;
        }
    }

    int queries(const uint32_t *r, const uint32_t *t, uint64_t n, tier::Query *send, uint64_t *counts) override {
        return guarded("two-tier queries", [&] {
            THIP(hipSetDevice(dev));
            w1_status_ok = false;
            set_requests(r, t, n, true);
            THIP(hipMemsetAsync(d_small, 0, 128 * 8, stream));
            THIP(hipMemsetAsync(d_small + kFirstBad, 0xFF, 8, stream));
            // requests read in place from pinned memory are staged into HBM by the count pass
            uint32_t *stage = n && in_place && !req_hbm ? (uint32_t *)d_req.ensure(8 * n) : nullptr;
            tier::launch_query_count(G, cur_r, cur_t, n, d_small + kCounts, d_small + kFirstBad, stage, stream);
            if (stage) {
                cur_r = stage;
                cur_t = stage + n;
            }
            THIP(hipMemcpyAsync(h_small, d_small, 129 * 8, hipMemcpyDeviceToHost, stream));
            THIP(hipStreamSynchronize(stream));
            uint64_t at = 0;
            for (uint32_t p = 0; p < G.world; p++) {
                counts[p] = h_small[kCounts + p];
                h_small[kCursor + p] = at;
                at += counts[p];
            }
            THIP(hipMemcpyAsync(d_small + kCursor, h_small + kCursor, 64 * 8, hipMemcpyHostToDevice, stream));
            // no wait: the exchange reads `send` on this stream (or copies it to the host here first)
            tier::launch_query_scatter(G, cur_r, cur_t, n, d_small + kCursor, send, stream);
            sent = send;
            sent_counts.assign(counts, counts + G.world);
        });
    }

    int reply_sizes(const tier::Query *recv, uint64_t n, const uint64_t *from, uint64_t *counts) override {
        return guarded("two-tier replies", [&] {
            THIP(hipSetDevice(dev));
            rq = recv;
            rq_n = n;
            uint64_t *lens = (uint64_t *)d_lens.ensure(8 * (n + 1));
            uint64_t *scr = (uint64_t *)d_scan.ensure(8 * (n / 1024 + 2));
            THIP(hipMemsetAsync(d_small + kBadQuery, 0xFF, 8, stream));
            tier::launch_reply_lengths(G, recv, n, lens, d_small + kBadQuery, stream,
                                       G.label ? (uint64_t *)d_srcb.ensure(8 * std::max<uint64_t>(n, 1)) : nullptr);
            tier::launch_scan(lens, n, scr, stream);
            // the offsets at the sources' boundaries: records per destination
            uint64_t at = 0;
            for (uint32_t p = 0; p <= G.world; p++) {
                THIP(hipMemcpyAsync(h_small + kCursor + p, lens + at, 8, hipMemcpyDeviceToHost, stream));
                if (p < G.world) at += from[p];
            }
            THIP(hipMemcpyAsync(h_small + kBadQuery, d_small + kBadQuery, 8, hipMemcpyDeviceToHost, stream));
            if (G.label) {  // the received segments' first queries, for launch_label_reply
                seg_firsts(from, kQs);
                THIP(hipMemcpyAsync(d_small + kQs, h_small + kQs, 8 * (G.world + 1), hipMemcpyHostToDevice, stream));
            }
            THIP(hipStreamSynchronize(stream));
            if (h_small[kBadQuery] != ~0ull)
                throw Error(KETOGPU_EINVAL, "a query for a node this rank does not own (query " +
                                                std::to_string(h_small[kBadQuery]) + ")");
            // label replies: the segment also carries one length per query
            for (uint32_t p = 0; p < G.world; p++)
                counts[p] = h_small[kCursor + p + 1] - h_small[kCursor + p] + (G.label ? from[p] : 0);
        });
    }

    // h_small[at + p] = items before segment p (p = 0..world)
    void seg_firsts(const uint64_t *cnt, size_t at) {
        uint64_t acc = 0;
        for (uint32_t p = 0; p < G.world; p++) {
            h_small[at + p] = acc;
            acc += cnt[p];
        }
        h_small[at + G.world] = acc;
    }

    uint64_t reply_unit() const override { return G.label ? 4 : sizeof(tier::Reply); }

    // World 1 through the exchange path's kernels with ONE host wait per step (plan label;
    // KETOGPU_TIER_ONE_WAIT=0: the general protocol).  With one owner the counts the
    // general protocol waits for are known or not needed: request i's queries take slots 2i
    // and 2i + 1 (no counting pass), the reply segment is the whole buffer, and the asker's
    // list lengths are the owner's (the same scan).  The reply buffer's capacity is the
    // last step's; a step whose replies outgrow it (known at the wait) is evaluated again
    // with a larger buffer.
    bool one_wait = true;  // KETOGPU_TIER_ONE_WAIT when the engine is made
    bool w1_status_ok = false;  // the status words are "none" (the last one-wait step reset them)
    bool has_world1() const override { return G.label && one_wait; }
    Buf d_q, d_rep;
    int step_world1(const uint32_t *r, const uint32_t *t, uint64_t n, uint64_t *bits, std::vector<uint32_t> &overflow,
                    uint64_t &reply_words) override {
        overflow.clear();
        return guarded("two-tier step", [&] {
            THIP(hipSetDevice(dev));
            set_requests(r, t, n, true);
            const uint64_t nq = 2 * n, words = (n + 63) / 64;
            tier::Query *q = (tier::Query *)d_q.ensure(sizeof(tier::Query) * std::max<uint64_t>(nq, 1));
            uint64_t *lens = (uint64_t *)d_lens.ensure(8 * (nq + 1));
            uint64_t *scr = (uint64_t *)d_scan.ensure(8 * (nq / 1024 + 2));
            uint64_t *allowed = (uint64_t *)d_bits.ensure(8 * std::max<uint64_t>(words, 1));
            uint4 *bnd = (uint4 *)d_bnd.ensure(16 * std::max<uint64_t>(n, 1));
            // first bad request, bad query: "none" — left so by the last one-wait step's emit
            if (!w1_status_ok) THIP(hipMemsetAsync(d_small + kFirstBad, 0xFF, 16, stream));
            w1_status_ok = false;
            uint32_t *stage = n && in_place && !req_hbm ? (uint32_t *)d_req.ensure(8 * n) : nullptr;
            tier::launch_query_pairs(G, cur_r, cur_t, n, q, d_small + kFirstBad, stage, stream);
            if (stage) {
                cur_r = stage;
                cur_t = stage + n;
            }
            uint64_t *srcb = (uint64_t *)d_srcb.ensure(8 * std::max<uint64_t>(nq, 1));
            tier::launch_reply_lengths(G, q, nq, lens, d_small + kBadQuery, stream, srcb);
            tier::launch_scan(lens, nq, scr, stream);
            const uint64_t *qs = (const uint64_t *)(d_small + kQs);  // (world 1: {0, nq}, not read)
            tier::Eval E{};
            E.roots = cur_r;
            E.targets = cur_t;
            E.n = n;
            E.allowed = allowed;
            E.stats = d_small + kStats;
            E.first_bad = d_small + kFirstBad;
            E.bnd = bnd;
            for (;;) {
                const uint64_t cap = d_rep.cap / 4;
                uint32_t *rep = (uint32_t *)d_rep.ensure(4 * std::max<uint64_t>(nq, 1));
                const uint64_t cap_now = std::max(cap, d_rep.cap / 4);
                // (the replies' pass also writes every request's bounds: one owner, one layout)
                tier::launch_label_reply(G, q, nq, lens, srcb, qs, 1, rep, cap_now, bnd, n, stream);
                THIP(hipEventRecord(ev0, stream));
                tier::launch_label_eval(G, E, rep, stream);
                THIP(hipEventRecord(ev1, stream));
                // answers (into pinned caller words in place, else one copy) and the status
                // words by one launch
                uint64_t *vbits = words ? (uint64_t *)host_view(bits, dev, false) : nullptr;
                tier::launch_emit(allowed, words, vbits, (unsigned long long *)d_small + kFirstBad, lens + nq,
                                  (unsigned long long *)d_hsmall + kFirstBad, d_hsmall + kLists, stream);
                if (words && !vbits) THIP(hipMemcpyAsync(bits, allowed, 8 * words, hipMemcpyDeviceToHost, stream));
                THIP(hipStreamSynchronize(stream));  // the step's one wait
                if (h_small[kBadQuery] != ~0ull)
                    throw Error(KETOGPU_EINVAL, "a query for a node this rank does not own (query " +
                                                    std::to_string(h_small[kBadQuery]) + ")");
                if (h_small[kFirstBad] != ~0ull)
                    throw Error(KETOGPU_EINVAL, "request " + std::to_string(h_small[kFirstBad]) +
                                                    " has an id outside the partitioned layout");
                reply_words = nq + h_small[kLists];
                if (reply_words >= (1ull << 32))
                    throw Error(KETOGPU_ENOMEM, "two-tier: a step's replies reach 2^32 words (" +
                                                    std::to_string(reply_words) + "); lower max_batch");
                if (reply_words <= cap_now) break;
                d_rep.ensure(4 * reply_words);  // outgrown: evaluate again with room for all of it
            }
            if (n) {
                float ms = 0;
                THIP(hipEventElapsedTime(&ms, ev0, ev1));
                eval_ms += ms;
                eval_launches++;
            }
            w1_status_ok = true;  // (the emit reset the status words)
            if (force_overflow) {
                std::fill(bits, bits + words, 0);
                for (uint64_t c = 0; c < n; c++) overflow.push_back((uint32_t)c);
            }
        });
    }
    void replies_from(const uint64_t *from, int world) override { recv_from.assign(from, from + world); }

    int reply_emit(tier::Reply *send, uint64_t cap) override {
        return guarded("two-tier replies", [&] {
            THIP(hipSetDevice(dev));
            if (G.label)
                tier::launch_label_reply(G, rq, rq_n, (const uint64_t *)d_lens.p, (const uint64_t *)d_srcb.p,
                                         (const uint64_t *)(d_small + kQs), G.world, (uint32_t *)send, cap, nullptr, 0,
                                         stream);
            else
                tier::launch_reply_copy(G, rq, rq_n, (const uint64_t *)d_lens.p, send, cap, stream);  // stream-ordered
        });
    }

    int evaluate(const uint32_t *r, const uint32_t *t, uint64_t n, const tier::Reply *recv, uint64_t nrecv, uint64_t *bits,
                 std::vector<uint32_t> &overflow) override {
        overflow.clear();
        return guarded("two-tier evaluation", [&] {
            THIP(hipSetDevice(dev));
            set_requests(r, t, n, recv == nullptr);
            const uint64_t words = (n + 63) / 64, units = (n + 15) / 16;
            uint64_t *allowed = (uint64_t *)d_bits.ensure(8 * std::max<uint64_t>(words, 1));
            uint32_t *lists[3];
            for (int k = 0; k < 3; k++) lists[k] = (uint32_t *)d_list[k].ensure(4 * std::max<uint64_t>(units, 1));
            w1_status_ok = false;
            if (!G.label) {  // (label: every unit stores its own answer word)
                THIP(hipMemsetAsync(allowed, 0, 8 * std::max<uint64_t>(words, 1), stream));
                THIP(hipMemsetAsync(d_small + kLists, 0, 6 * 8, stream));
            }
            if (!recv) THIP(hipMemsetAsync(d_small + kFirstBad, 0xFF, 8, stream));
            tier::Eval E{};
            E.roots = cur_r;
            E.targets = cur_t;
            E.n = n;
            E.allowed = allowed;
            E.stats = d_small + kStats;
            E.first_bad = d_small + kFirstBad;
            if (recv && !G.label) {
                // seed bounds are u32 offsets into the received entries (tier_seed_kernel): a
                // step past 2^32 entries fails on this rank (the code travels in the next
                // status gather); a smaller ketogpu_tier_opts.max_batch splits it
                if (nrecv >= (1ull << 32))
                    throw Error(KETOGPU_ENOMEM, "two-tier: a step received 2^32 or more reply entries (" +
                                                    std::to_string(nrecv) + "); lower max_batch");
                uint4 *bnd = (uint4 *)d_bnd.ensure(16 * std::max<uint64_t>(n, 1));
                THIP(hipMemsetAsync(bnd, 0, 16 * std::max<uint64_t>(n, 1), stream));
                tier::Rec *seed = (tier::Rec *)d_seed.ensure(sizeof(tier::Rec) * std::max<uint64_t>(nrecv, 1));
                tier::launch_seed_records(G, recv, nrecv, seed, bnd, n, stream);
                E.bnd = bnd;
                E.recv = seed;
                E.recv_base_f = (int64_t)((intptr_t)seed - (intptr_t)G.core_f) / (int64_t)sizeof(tier::Rec);
                E.recv_base_b = (int64_t)((intptr_t)seed - (intptr_t)G.core_b) / (int64_t)sizeof(tier::Rec);
            }
            if (G.label) {  // one intersection per request, nothing left for a later stage
                const uint32_t *rwords = (const uint32_t *)recv;
                if (recv) {
                    if (nrecv >= (1ull << 32))
                        throw Error(KETOGPU_ENOMEM, "two-tier: a step received 2^32 or more reply words (" +
                                                        std::to_string(nrecv) + "); lower max_batch");
                    if (sent_counts.size() != G.world || recv_from.size() != G.world)
                        throw Error(KETOGPU_EINVAL, "two-tier: label replies without this step's queries");
                    uint64_t nsent = 0;
                    for (uint64_t c : sent_counts) nsent += c;
                    seg_firsts(sent_counts.data(), kSq);
                    seg_firsts(recv_from.data(), kRp);
                    THIP(hipMemcpyAsync(d_small + kSq, h_small + kSq, 8 * 144, hipMemcpyHostToDevice, stream));
                    uint64_t *lens = (uint64_t *)d_lens.ensure(8 * (nsent + 1));
                    uint64_t *scr = (uint64_t *)d_scan.ensure(8 * (nsent / 1024 + 2));
                    const uint64_t *sq = (const uint64_t *)(d_small + kSq), *rp = (const uint64_t *)(d_small + kRp);
                    tier::launch_label_lens(rwords, nsent, sq, rp, G.world, lens, stream);
                    tier::launch_scan(lens, nsent, scr, stream);
                    uint4 *bnd = (uint4 *)d_bnd.ensure(16 * std::max<uint64_t>(n, 1));
                    THIP(hipMemsetAsync(bnd, 0, 16 * std::max<uint64_t>(n, 1), stream));
                    tier::launch_label_bounds(sent, nsent, sq, lens, G.world, bnd, n, nrecv, stream);
                    E.bnd = bnd;
                }
                THIP(hipEventRecord(ev0, stream));
                tier::launch_label_eval(G, E, rwords, stream);
                THIP(hipEventRecord(ev1, stream));
                if (words) THIP(hipMemcpyAsync(bits, allowed, 8 * words, hipMemcpyDeviceToHost, stream));
                THIP(hipMemcpyAsync(h_small + kFirstBad, d_small + kFirstBad, 8, hipMemcpyDeviceToHost, stream));
                THIP(hipStreamSynchronize(stream));
                if (n) {
                    float ms = 0;
                    THIP(hipEventElapsedTime(&ms, ev0, ev1));
                    eval_ms += ms;
                    eval_launches++;
                }
                if (h_small[kFirstBad] != ~0ull)
                    throw Error(KETOGPU_EINVAL, "request " + std::to_string(h_small[kFirstBad]) +
                                                    " has an id outside the partitioned layout");
                if (force_overflow) {
                    std::fill(bits, bits + words, 0);
                    for (uint64_t c = 0; c < n; c++) overflow.push_back((uint32_t)c);
                }
                return;
            }
            unsigned *lc = (unsigned *)(d_small + kLists);  // three u32 list counts (+ padding)
            THIP(hipEventRecord(ev0, stream));
            tier::launch_eval(0, G, E, nullptr, nullptr, lists[0], lc + 0, 0, stream);
            THIP(hipEventRecord(ev1, stream));
            for (int s = 1; s < tier::kStages; s++)
                tier::launch_eval(s, G, E, lists[s - 1], lc + (s - 1), lists[s], lc + s,
                                  (unsigned)(n_cu * tier::stage_units_per_cu(s)), stream);
            if (words) THIP(hipMemcpyAsync(bits, allowed, 8 * words, hipMemcpyDeviceToHost, stream));
            THIP(hipMemcpyAsync(h_small + kFirstBad, d_small + kFirstBad, 8 * 4, hipMemcpyDeviceToHost, stream));
            THIP(hipStreamSynchronize(stream));
            if (n) {
                float ms = 0;
                THIP(hipEventElapsedTime(&ms, ev0, ev1));
                eval_ms += ms;
                eval_launches++;
            }
            if (h_small[kFirstBad] != ~0ull)
                throw Error(KETOGPU_EINVAL, "request " + std::to_string(h_small[kFirstBad]) +
                                                " has an id outside the partitioned layout");
            if (force_overflow) {
                std::fill(bits, bits + words, 0);
                for (uint64_t c = 0; c < n; c++) overflow.push_back((uint32_t)c);
                return;
            }
            const uint32_t *hc = (const uint32_t *)(h_small + kLists);
            const uint32_t last = hc[tier::kStages - 1];
            if (last) {  // units no table held: their requests go to the per-level engine
                std::vector<uint32_t> u(last);
                THIP(hipMemcpy(u.data(), lists[tier::kStages - 1], 4 * (uint64_t)last, hipMemcpyDeviceToHost));
                for (uint32_t x : u)
                    for (uint64_t c = (uint64_t)x * 16; c < std::min<uint64_t>(n, (uint64_t)x * 16 + 16); c++)
                        overflow.push_back((uint32_t)c);
            }
        });
    }

    void stats(ketogpu_tier_stats &st) override {
        if (!d_small) return;
        std::vector<uint64_t> s(kEvalStatsLen);
        if (hipMemcpy(s.data(), d_small + kStats, 8 * kEvalStatsLen, hipMemcpyDeviceToHost) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        uint64_t rows = 0, edges = 0;
        for (size_t k = 0; k < 1024; k++) rows += s[8 + 4 * k], edges += s[8 + 4 * k + 1];
        st.rows_opened = rows;
        st.records_read = edges;
        st.core_records = core_records;
        st.seed_records = seed_records;
        st.eval_kernel_ms = eval_ms;
        st.eval_kernel_launches = eval_launches;
        st.label = G.label;
        st.label_words = label_words;
        st.label_build_ms = label_ms;
    }

    std::string error() override { return err; }
};

}  // namespace

// ------------------------------------------------------------------ engine
struct ketogpu_tier {
    std::unique_ptr<TierSteps> steps;
    ketogpu_comm *chandle = nullptr;  // borrowed
    Comm *comm = nullptr;
    int rank = 0, world = 1;
    uint64_t max_batch = 4u << 20;
    uint64_t fallback_bytes = 2ull << 30;
    const ketogpu_shard *shard = nullptr;
    int device = -1;
    // exchange buffers: in the steps' memory, and host staging when the transport is host
    // memory while the steps are device memory
    Buf q_send, q_recv, r_send, r_recv, h_send, h_recv;
    bool stage = false;
    Buf small_d;  // count all-gathers on an RCCL communicator
    std::vector<uint64_t> mat;
    // the per-level engine for requests no LDS table held (built on first need, collectively)
    ketogpu_part *part = nullptr;
    ketogpu_part_engine *pe = nullptr;
    std::mutex mu;
    ketogpu_tier_stats st{};

    uint64_t *h_gather = nullptr;  // pinned staging of the count all-gathers (RCCL)
    static constexpr size_t kGatherMax = 80;  // values per rank (at most world + 1 = 65)

    ~ketogpu_tier() {
        if (pe) ketogpu_part_engine_free(pe);
        if (part) ketogpu_part_free(part);
        if (h_gather) {
            (void)hipStreamSynchronize(stream());
            (void)hipHostFree(h_gather);
        }
    }

    hipStream_t stream() const { return steps->stream; }

    // every rank's n u64 values -> mat (world * n, rank order)
    void gather(const uint64_t *v, size_t n) {
        mat.assign(n * world, 0);
        if (!comm || (world == 1 && !comm->loop_self)) {  // a gather over one rank is the identity
            std::copy(v, v + n, mat.begin());
            return;
        }
        const auto t0 = Clock::now();
        if (comm->device) {
            // through pinned staging: both copies are asynchronous DMA, one wait
            if (n > kGatherMax) throw Error(KETOGPU_EINVAL, "two-tier: gather wider than its staging");
            if (!h_gather)
                THIP(hipHostMalloc((void **)&h_gather, 8 * kGatherMax * (world + 1), hipHostMallocDefault));
            uint64_t *d = (uint64_t *)small_d.ensure(8 * n * (world + 1));
            std::copy(v, v + n, h_gather);
            THIP(hipMemcpyAsync(d, h_gather, n * 8, hipMemcpyHostToDevice, stream()));
            comm->allgather(d, d + n, n * 8, stream());
            THIP(hipMemcpyAsync(h_gather + n, d + n, n * world * 8, hipMemcpyDeviceToHost, stream()));
            THIP(hipStreamSynchronize(stream()));
            std::copy(h_gather + n, h_gather + n + n * world, mat.begin());
        } else {
            comm->allgather(v, mat.data(), n * 8, stream());
        }
        st.collectives++;
        st.exchange_ms += ms_since(t0);
    }

    // counts[world] items of `unit` bytes grouped by destination in `send` -> `recv` grouped
    // by source (grown to fit), *n_in items; from[world] items per source.  The status of
    // the step before travels with the counts: the agreed (largest) code is returned.
    int exchange(int code, const uint64_t *counts, uint64_t unit, Buf &send, Buf &recv, uint64_t *n_in,
                 std::vector<uint64_t> &from) {
        const size_t W1 = (size_t)world + 1;
        std::vector<uint64_t> mine(W1, 0);
        if (!code) std::copy(counts, counts + world, mine.begin());
        mine[world] = (uint64_t)code;
        gather(mine.data(), W1);
        int agreed = 0;
        for (int r = 0; r < world; r++) agreed = std::max(agreed, (int)mat[r * W1 + world]);
        *n_in = 0;
        from.assign(world, 0);
        if (agreed) return agreed;
        std::vector<uint64_t> sb(world), rb(world);
        uint64_t ns = 0, nr = 0;
        for (int p = 0; p < world; p++) {
            from[p] = mat[(size_t)p * W1 + rank];
            sb[p] = unit * mat[(size_t)rank * W1 + p];
            rb[p] = unit * from[p];
            ns += sb[p];
            nr += rb[p];
        }
        const auto t0 = Clock::now();
        if (world == 1 && !comm->loop_self && !stage) {
            // one rank: what it sends is what it receives, the buffers trade places (no copy)
            std::swap(send.p, recv.p);
            std::swap(send.cap, recv.cap);
            st.collectives++;
            st.exchange_ms += ms_since(t0);
            *n_in = nr / unit;
            return KETOGPU_OK;
        }
        recv.ensure(nr);
        if (stage) {  // device steps, host transport
            h_send.ensure(ns);
            h_recv.ensure(nr);
            if (ns) THIP(hipMemcpyAsync(h_send.p, send.p, ns, hipMemcpyDeviceToHost, stream()));
            THIP(hipStreamSynchronize(stream()));
            comm->alltoallv(h_send.p, sb.data(), h_recv.p, rb.data(), stream());
            if (nr) THIP(hipMemcpyAsync(recv.p, h_recv.p, nr, hipMemcpyHostToDevice, stream()));
            THIP(hipStreamSynchronize(stream()));
        } else {
            // RCCL: on the steps' stream, ordered before the next step's kernels (no wait)
            comm->alltoallv(send.p, sb.data(), recv.p, rb.data(), stream());
        }
        st.collectives++;
        st.exchange_ms += ms_since(t0);
        *n_in = nr / unit;
        return KETOGPU_OK;
    }

    [[noreturn]] void fail(int code, int local, const std::string &why) {
        throw Error(code, local == code && !why.empty() ? why : "two-tier: a step failed on another rank");
    }

    // one step of at most max_batch requests of this rank (n may be 0)
    void step(const uint32_t *roots, const uint32_t *targets, uint64_t n, uint64_t *bits) {
        st.batches++;
        std::vector<uint32_t> overflow;
        std::fill(bits, bits + (n + 63) / 64, 0);
        int local = 0;
        const auto t_eval = Clock::now();
        double exch0 = st.exchange_ms;
        if (!comm) {
            local = steps->evaluate(roots, targets, n, nullptr, 0, bits, overflow);
            if (local) throw Error(local, steps->error());
        } else if (world == 1 && !comm->loop_self && !stage && steps->has_world1()) {
            uint64_t words = 0;  // one rank: nothing to agree on, the exchange is the identity
            local = steps->step_world1(roots, targets, n, bits, overflow, words);
            if (local) throw Error(local, steps->error());
            st.queries_sent += 2 * n;
            st.records_sent += words;
            st.records_received += words;
        } else {
            std::vector<uint64_t> counts(world, 0), from;
            q_send.ensure(sizeof(tier::Query) * 2 * std::max<uint64_t>(n, 1));
            local = steps->queries(roots, targets, n, q_send.as<tier::Query>(), counts.data());
            if (!local)
                for (uint64_t c : counts) st.queries_sent += c;
            uint64_t nq = 0, nr = 0;
            int code = exchange(local, counts.data(), sizeof(tier::Query), q_send, q_recv, &nq, from);
            if (code) fail(code, local, steps->error());
            local = steps->reply_sizes(q_recv.as<tier::Query>(), nq, from.data(), counts.data());
            uint64_t out = 0;
            const uint64_t unit = steps->reply_unit();
            if (!local) {
                for (uint64_t c : counts) out += c;
                try {
                    r_send.ensure(unit * out);
                } catch (const Error &e) {
                    local = e.code;
                }
            }
            if (!local) local = steps->reply_emit(r_send.as<tier::Reply>(), out);
            if (!local) st.records_sent += out;
            code = exchange(local, counts.data(), unit, r_send, r_recv, &nr, from);
            if (code) fail(code, local, steps->error());
            steps->replies_from(from.data(), world);
            st.records_received += nr;
            local = steps->evaluate(roots, targets, n, r_recv.as<tier::Reply>(), nr, bits, overflow);
        }
        st.evaluate_ms += ms_since(t_eval) - (st.exchange_ms - exch0);
        // every rank's status and unfinished requests (world 1: its own)
        uint64_t v[2] = {(uint64_t)local, local ? 0 : (uint64_t)overflow.size()};
        gather(v, 2);
        int agreed = 0;
        uint64_t total = 0;
        std::vector<uint64_t> over(world);
        for (int r = 0; r < world; r++) {
            agreed = std::max(agreed, (int)mat[2 * r]);
            over[r] = mat[2 * r + 1];
            total += over[r];
        }
        if (agreed) fail(agreed, local, steps->error());
        if (total) fallback(roots, targets, overflow, over, total, bits);
    }

    // the largest status code of every rank (0: all succeeded)
    int agree(int rc) {
        if (!comm || world == 1) return rc;
        HostColl hc(comm);
        st.collectives++;
        return hc.agree(rc);
    }
    void drop_fallback() {
        if (pe) ketogpu_part_engine_free(pe);
        if (part) ketogpu_part_free(part);
        pe = nullptr;
        part = nullptr;
    }

    // requests no LDS table held: every rank's, gathered, answered by the per-level engine
    // (which takes the same requests on every rank), each rank keeping its own answers
    void fallback(const uint32_t *roots, const uint32_t *targets, const std::vector<uint32_t> &mine,
                  const std::vector<uint64_t> &over, uint64_t total, uint64_t *bits) {
        if (!shard) throw Error(KETOGPU_EINVAL, "two-tier: requests outgrew the host steps' tables");
        st.fallback_calls++;
        st.overflow_requests += mine.size();
        std::vector<uint32_t> pairs(2 * mine.size());
        std::vector<uint32_t> hr, ht;  // requests in device memory: a host copy for this rare path
        if (steps->device && !mine.empty() && device_memory(roots)) {
            const uint64_t n = (uint64_t)mine.back() + 1;
            hr.resize(n);
            ht.resize(n);
            THIP(hipMemcpy(hr.data(), roots, 4 * n, hipMemcpyDefault));
            THIP(hipMemcpy(ht.data(), targets, 4 * n, hipMemcpyDefault));
            roots = hr.data();
            targets = ht.data();
        }
        for (size_t k = 0; k < mine.size(); k++) {
            pairs[2 * k] = roots[mine[k]];
            pairs[2 * k + 1] = targets[mine[k]];
        }
        std::vector<uint32_t> all(2 * total);
        if (comm) {
            HostColl hc(comm);
            std::vector<uint64_t> sizes;
            std::vector<char> got = hc.allgatherv(pairs.data(), pairs.size() * 4, &sizes);
            if (got.size() != all.size() * 4) throw Error(KETOGPU_EDEVICE, "two-tier: overflow gather size mismatch");
            memcpy(all.data(), got.data(), got.size());
            st.collectives += 2;
        } else {
            all = pairs;
        }
        std::vector<uint32_t> r(total), t(total);
        for (uint64_t k = 0; k < total; k++) r[k] = all[2 * k], t[k] = all[2 * k + 1];
        if (!pe) {  // collective: every rank reaches this in the same step
            ketogpu_part_opts po{};
            po.device = device;
            po.rank = rank;
            po.world = world;
            po.record_capacity = 1 << 22;
            po.max_words_per_round = 256;
            po.state_budget_bytes = fallback_bytes;
            // each construction's status is agreed before the next collective: a rank whose
            // device state does not fit (free HBM differs between ranks) fails every rank
            // alike instead of leaving its peers in the engine's init gather
            int rc = ketogpu_part_new(shard, &po, &part);
            std::string why = rc ? std::string(ketogpu_last_error()) : std::string();
            if (const int a = agree(rc)) {
                drop_fallback();
                throw Error(a, rc == a ? why : "two-tier: the fallback engine failed on another rank");
            }
            ketogpu_part_engine_opts eo{};
            eo.direction = KETOGPU_PART_AUTO;
            rc = ketogpu_part_engine_new(part, chandle, &eo, &pe);
            why = rc ? std::string(ketogpu_last_error()) : std::string();
            if (const int a = agree(rc)) {
                drop_fallback();
                throw Error(a, rc == a ? why : "two-tier: the fallback engine failed on another rank");
            }
        }
        std::vector<uint64_t> ans((total + 63) / 64, 0);
        if (const int rc = ketogpu_part_check_ids(pe, r.data(), t.data(), total, ans.data()))
            throw Error(rc, ketogpu_last_error());
        uint64_t at = 0;
        for (int p = 0; p < rank; p++) at += over[p];
        for (size_t k = 0; k < mine.size(); k++) {
            const uint64_t j = at + k;
            if ((ans[j >> 6] >> (j & 63)) & 1ull) bits[mine[k] >> 6] |= 1ull << (mine[k] & 63);
        }
    }

    void check_ids(const uint32_t *roots, const uint32_t *targets, uint64_t n, uint64_t *bits) {
        if (steps->device) THIP(hipSetDevice(steps->dev));
        st.calls++;
        st.requests += n;
        // every rank runs the same number of steps (the largest batch decides)
        uint64_t nsteps = (n + max_batch - 1) / max_batch;
        if (comm) {
            gather(&nsteps, 1);
            for (int r = 0; r < world; r++) nsteps = std::max(nsteps, mat[r]);
        }
        std::vector<uint64_t> tmp;
        for (uint64_t s = 0; s < nsteps; s++) {
            const uint64_t b = std::min(n, s * max_batch), e = std::min(n, b + max_batch);
            if (b % 64 == 0) {
                step(roots + b, targets + b, e - b, bits + b / 64);
            } else {  // unreachable: max_batch is a multiple of 64
                tmp.assign((e - b + 63) / 64, 0);
                step(roots + b, targets + b, e - b, tmp.data());
            }
        }
    }

    void init(std::unique_ptr<TierSteps> s, ketogpu_comm *c, const ketogpu_tier_opts *o) {
        steps = std::move(s);
        chandle = c;
        comm = c ? c->c.get() : nullptr;
        rank = comm ? comm->rank : 0;
        world = comm ? comm->world : 1;
        if (o && o->max_batch) max_batch = std::max<uint64_t>(64, o->max_batch / 64 * 64);
        max_batch = std::min<uint64_t>(max_batch, 1ull << 30);  // tags hold request << 1 in 32 bits
        if (o && o->fallback_state_bytes) fallback_bytes = o->fallback_state_bytes;
        if (comm && comm->device && (!steps->device || comm->dev != steps->dev))
            throw Error(KETOGPU_EINVAL, "two-tier: an RCCL communicator needs device steps on its device");
        stage = comm && steps->device && !comm->device;
        for (Buf *b : {&q_send, &q_recv, &r_send, &r_recv}) {
            b->device = steps->device;
            b->dev = steps->dev;
        }
        small_d.device = comm && comm->device;
        small_d.dev = comm ? comm->dev : -1;
    }
};

#define TAPI_BEGIN try {
#define TAPI_END                                                                                       \
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

int ketogpu_core_gather(const ketogpu_shard *s, ketogpu_comm *comm, uint64_t core_budget_bytes, ketogpu_core **out) {
    TAPI_BEGIN
    if (!s || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    ketogpu_shard_graph v{};
    int rc = ketogpu_shard_view(s, &v);
    std::string why = rc ? std::string(ketogpu_last_error()) : std::string();
    Comm *c = comm ? comm->c.get() : nullptr;
    if (c && c->world != (int)(rc ? c->world : (int)v.world))
        throw Error(KETOGPU_EINVAL, "two-tier: the communicator's world differs from the shard's");
    if (c && c->world > 1) {  // a rank whose shard is not ready fails every rank alike
        HostColl hc(c);
        const int a = hc.agree(rc);
        if (a) throw Error(a, rc == a ? why : "two-tier: loading failed on another rank");
    } else if (rc) {
        throw Error(rc, why);
    }
    if (!c && v.world != 1) throw Error(KETOGPU_EINVAL, "two-tier: a shard of several ranks needs a communicator");
    *out = gather_core(v, c, core_budget_bytes).release();
    TAPI_END
}

int ketogpu_core_get_view(const ketogpu_core *c, ketogpu_core_view *out) {
    TAPI_BEGIN
    if (!c || !out) throw Error(KETOGPU_EINVAL, "null argument");
    out->num_interior = (uint32_t)c->Ni;
    out->f_off = c->f_off.data();
    out->f_col = c->f_col.data();
    out->b_off = c->b_off.data();
    out->b_col = c->b_col.data();
    out->bytes = c->bytes();
    TAPI_END
}

void ketogpu_core_free(ketogpu_core *c) { delete c; }

int ketogpu_tier_new(const ketogpu_shard *s, const ketogpu_core *core, ketogpu_comm *comm,
                     const ketogpu_tier_opts *opts, ketogpu_tier **out) {
    TAPI_BEGIN
    if (!s || !core || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto d = std::make_unique<TierDevice>();
    const int device = opts ? opts->device : 0;
    d->init(s, core, device);
    if (comm && comm->c->world != (int)d->G.world)
        throw Error(KETOGPU_EINVAL, "two-tier: the communicator's world differs from the shard's");
    if (!comm && d->G.world != 1) throw Error(KETOGPU_EINVAL, "two-tier: a shard of several ranks needs a communicator");
    auto t = std::make_unique<ketogpu_tier>();
    t->shard = s;
    t->device = device;
    t->init(std::move(d), comm, opts);
    *out = t.release();
    TAPI_END
}

int ketogpu_tier_new_steps(const ketogpu_tier_steps *steps, ketogpu_comm *comm, const ketogpu_tier_opts *opts,
                           ketogpu_tier **out) {
    TAPI_BEGIN
    if (!steps || !out || !steps->queries || !steps->reply_sizes || !steps->reply_emit || !steps->evaluate)
        throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto s = std::make_unique<VtableTier>();
    s->v = *steps;
    auto t = std::make_unique<ketogpu_tier>();
    t->init(std::move(s), comm, opts);
    *out = t.release();
    TAPI_END
}

int ketogpu_tier_check_ids(ketogpu_tier *t, const uint32_t *roots, const uint32_t *targets, size_t n,
                           uint64_t *allowed_bits) {
    TAPI_BEGIN
    if (!t || (n && (!roots || !targets || !allowed_bits))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(t->mu);
    t->check_ids(roots, targets, n, allowed_bits);
    TAPI_END
}

int ketogpu_tier_stats_get(ketogpu_tier *t, ketogpu_tier_stats *out) {
    TAPI_BEGIN
    if (!t || !out) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(t->mu);
    *out = t->st;
    t->steps->stats(*out);
    TAPI_END
}

void ketogpu_tier_free(ketogpu_tier *t) { delete t; }

}  // extern "C"
