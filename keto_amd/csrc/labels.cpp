// labels.cpp — builds plan "label"'s 2-hop reachability labels and head arrays (labels.hpp).
#include "labels.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <shared_mutex>

#include "core_index.hpp"  // build_threads, parallel_chunks

namespace ketogpu {

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

// the interior graph in both directions: forward fint(v), backward the interior prefix of
// the sorted rev(v) (the nodes of a path between interior nodes are all interior).  On a
// writable snapshot rows end in placeholder slots (Df / Dbi, the two largest interior ids,
// snapshot_write.cpp make_writable): the real interior entries are those below Dbi.
struct IAdj {
    const uint32_t *col[2] = {nullptr, nullptr};
    std::vector<uint64_t> beg[2];
    std::vector<uint32_t> deg[2];
};

void make_adj(const Snapshot &s, IAdj &a) {
    const uint32_t n = s.Ni, bound = s.writable ? s.Dbi : n;
    a.col[0] = s.fint_col.data();
    a.col[1] = s.rev_col.data();
    for (int d = 0; d < 2; d++) {
        a.beg[d].resize(n);
        a.deg[d].resize(n);
    }
    parallel_chunks(n, 1 << 16, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t v = b; v < e; v++) {
            const uint32_t *fb = s.fint_col.data() + s.fint_off[v], *fe = s.fint_col.data() + s.fint_off[v + 1];
            a.beg[0][v] = s.fint_off[v];
            a.deg[0][v] = s.writable ? (uint32_t)(std::lower_bound(fb, fe, bound) - fb) : (uint32_t)(fe - fb);
            const uint32_t *rb = s.rev_col.data() + s.rev_off[v], *re = s.rev_col.data() + s.rev_off[v + 1];
            a.beg[1][v] = s.rev_off[v];
            a.deg[1][v] = (uint32_t)(std::lower_bound(rb, re, bound) - rb);
        }
    });
}

// a topological order of the interior graph (forward edges), or false when it has a cycle
bool topo_order(const IAdj &a, std::vector<uint32_t> &topo) {
    const uint32_t n = (uint32_t)a.deg[0].size();
    std::vector<uint32_t> indeg(a.deg[1].begin(), a.deg[1].end());
    topo.clear();
    topo.reserve(n);
    for (uint32_t v = 0; v < n; v++)
        if (!indeg[v]) topo.push_back(v);
    for (size_t h = 0; h < topo.size(); h++) {
        const uint32_t y = topo[h];
        const uint32_t *c = a.col[0] + a.beg[0][y];
        for (uint32_t j = 0; j < a.deg[0][y]; j++)
            if (--indeg[c[j]] == 0) topo.push_back(c[j]);
    }
    return topo.size() == n;
}

// M[v] bit i = landmark order[i] reaches v along direction d (reflexive).  An acyclic
// interior graph (topo non-empty): one pass in topological order (reverse order backward);
// else a frontier propagation of 64-bit masks, level by level, on every build thread
void reach_masks(const IAdj &a, const std::vector<uint32_t> &order, const std::vector<uint32_t> &topo, uint32_t bits,
                 int d, std::vector<uint64_t> &M) {
    const uint32_t n = (uint32_t)order.size();
    if (!topo.empty()) {
        M.assign(n, 0);
        for (uint32_t i = 0; i < bits; i++) M[order[i]] |= 1ull << i;
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t y = topo[d == 0 ? k : n - 1 - k];
            const uint64_t m = M[y];
            if (!m) continue;
            const uint32_t *c = a.col[d] + a.beg[d][y];
            for (uint32_t j = 0; j < a.deg[d][y]; j++) M[c[j]] |= m;
        }
        return;
    }
    std::vector<std::atomic<uint64_t>> A(n), P(n);
    std::vector<std::atomic<uint8_t>> inq(n);
    parallel_chunks(n, 1 << 16, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t v = b; v < e; v++) {
            A[v].store(0, std::memory_order_relaxed);
            P[v].store(0, std::memory_order_relaxed);
            inq[v].store(0, std::memory_order_relaxed);
        }
    });
    std::vector<uint32_t> F;
    for (uint32_t i = 0; i < bits; i++) {
        const uint32_t w = order[i];
        A[w].fetch_or(1ull << i);
        P[w].fetch_or(1ull << i);
        if (!inq[w].exchange(1)) F.push_back(w);
    }
    const int T = build_threads();
    std::vector<std::vector<uint32_t>> nxt(T);
    while (!F.empty()) {
        parallel_chunks(F.size(), 256, [&](int tid, uint64_t b, uint64_t e) {
            for (uint64_t k = b; k < e; k++) {
                const uint32_t y = F[k];
                inq[y].store(0);
                const uint64_t dl = P[y].exchange(0);
                if (!dl) continue;
                const uint32_t *c = a.col[d] + a.beg[d][y];
                for (uint32_t j = 0; j < a.deg[d][y]; j++) {
                    const uint32_t z = c[j];
                    const uint64_t nw = dl & ~A[z].fetch_or(dl);
                    if (!nw) continue;
                    P[z].fetch_or(nw);
                    if (!inq[z].exchange(1)) nxt[tid].push_back(z);
                }
            }
        });
        F.clear();
        for (auto &x : nxt) {
            F.insert(F.end(), x.begin(), x.end());
            x.clear();
        }
    }
    M.resize(n);
    parallel_chunks(n, 1 << 16, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t v = b; v < e; v++) M[v] = A[v].load(std::memory_order_relaxed);
    });
}

// one build thread's search state: visit and mark stamps (landmark rank r, direction d:
// stamp 2r + 1 + d, never 0), the queue, and the entries found in a parallel batch
struct Searcher {
    std::vector<uint32_t> vis, mark, q;
    // (node, rank) per direction, bucketed by node % threads (the merge thread of the node)
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> add[2];
};

}  // namespace

namespace {
void build_reach(IAdj &a, uint32_t n, ReachLabels &out);
}

void build_reach_labels(const Snapshot &s, ReachLabels &out) {
    out = ReachLabels{};
    IAdj a;
    make_adj(s, a);
    build_reach(a, s.Ni, out);
}

void copy_interior(const Snapshot &s, InteriorCsr &out) {
    IAdj a;
    make_adj(s, a);
    const uint32_t n = s.Ni;
    out.n = n;
    for (int d = 0; d < 2; d++) {
        std::vector<uint64_t> &off = d == 0 ? out.f_off : out.b_off;
        std::vector<uint32_t> &col = d == 0 ? out.f_col : out.b_col;
        off.assign((size_t)n + 1, 0);
        for (uint32_t v = 0; v < n; v++) off[v + 1] = off[v] + a.deg[d][v];
        col.resize(off[n]);
        parallel_chunks(n, 1 << 14, [&](int, uint64_t b, uint64_t e) {
            for (uint64_t v = b; v < e; v++)
                std::copy(a.col[d] + a.beg[d][v], a.col[d] + a.beg[d][v] + a.deg[d][v], col.begin() + (ptrdiff_t)off[v]);
        });
    }
}

void build_reach_labels_csr(uint32_t n, const uint64_t *f_off, const uint32_t *f_col, const uint64_t *b_off,
                            const uint32_t *b_col, ReachLabels &out) {
    out = ReachLabels{};
    IAdj a;
    a.col[0] = f_col;
    a.col[1] = b_col;
    for (int d = 0; d < 2; d++) {
        const uint64_t *off = d == 0 ? f_off : b_off;
        a.beg[d].assign(off, off + n);
        a.deg[d].resize(n);
        for (uint32_t v = 0; v < n; v++) a.deg[d][v] = (uint32_t)(off[v + 1] - off[v]);
    }
    build_reach(a, n, out);
}

namespace {
void build_reach(IAdj &a, uint32_t n, ReachLabels &out) {
    const auto t0 = Clock::now();
    out.n = n;
    if (!n) return;
    // the searches' stamps 2r + 1 + d are u32: past 2^31 - 1 interior nodes they would wrap
    // onto earlier stamps (a node would look visited, a search pruned) — refused instead
    if (n >= 0x7FFFFFFFu) throw Error(KETOGPU_EINVAL, "plan label: 2^31 or more interior nodes");
    // rank: most central first ((interior out-degree + 1) x (interior in-degree + 1))
    out.order.resize(n);
    std::iota(out.order.begin(), out.order.end(), 0u);
    {  // (key descending, node ascending) as one u64 per node: ~key << 32 | node
        std::vector<uint64_t> kv(n);
        for (uint32_t v = 0; v < n; v++) {
            const uint64_t key = std::min<uint64_t>((uint64_t)(a.deg[0][v] + 1) * (a.deg[1][v] + 1), 0xFFFFFFFFull);
            kv[v] = (0xFFFFFFFFull - key) << 32 | v;
        }
        std::sort(kv.begin(), kv.end());
        for (uint32_t k = 0; k < n; k++) out.order[k] = (uint32_t)kv[k];
    }
    static const bool plog = getenv("KETOGPU_LABEL_LOG") != nullptr;
    auto phase = [&](const char *what) {
        if (plog) fprintf(stderr, "[pll] %-12s %8.1f ms\n", what, ms_since(t0));
    };
    phase("order");
    const uint32_t bits = std::min<uint32_t>(n, kMaskBits);
    out.bits = bits;
    std::vector<uint32_t> topo;
    if (!topo_order(a, topo)) topo.clear();
    reach_masks(a, out.order, topo, bits, 0, out.min);
    reach_masks(a, out.order, topo, bits, 1, out.mout);
    phase("masks");
    // pruned searches of the other landmarks; L[0] = Lin, L[1] = Lout (ranks, unsorted
    // while building: the coverage test marks one side and scans the other)
    std::vector<std::vector<uint32_t>> L[2];
    L[0].resize(n);
    L[1].resize(n);
    const int T = build_threads();
    std::vector<Searcher> sr(T);
    for (auto &x : sr) {
        x.vis.assign(n, 0);
        x.mark.assign(n, 0);
        x.add[0].resize(T);
        x.add[1].resize(T);
    }
    const std::vector<uint64_t> *mask[2] = {&out.min, &out.mout};
    // d = 0: forward from w, entries into Lin (w ->* y); d = 1: backward, into Lout.  The
    // search prunes at y when the labels so far answer the pair (w, y) (d = 0: Lout(w) meets
    // Lin(y), or mout(w) meets min(y)); direct = false: entries go to the searcher's list
    auto search = [&](Searcher &S, uint32_t r, int d, bool direct) {
        const uint32_t w = out.order[r], st = 2 * r + 1 + (uint32_t)d;
        for (uint32_t x : L[d ^ 1][w]) S.mark[x] = st;
        const uint64_t wm = (*mask[d ^ 1])[w];
        const std::vector<uint64_t> &ym = *mask[d];
        S.q.clear();
        S.q.push_back(w);
        S.vis[w] = st;
        for (size_t h = 0; h < S.q.size(); h++) {
            const uint32_t y = S.q[h];
            if (wm & ym[y]) continue;
            bool cov = false;
            for (uint32_t x : L[d][y])
                if (S.mark[x] == st) {
                    cov = true;
                    break;
                }
            if (cov) continue;
            if (direct)
                L[d][y].push_back(r);
            else
                S.add[d][y % (uint32_t)T].push_back({y, r});
            const uint32_t *c = a.col[d] + a.beg[d][y];
            for (uint32_t j = 0; j < a.deg[d][y]; j++) {
                const uint32_t z = c[j];
                if (S.vis[z] != st) {
                    S.vis[z] = st;
                    S.q.push_back(z);
                }
            }
        }
    };
    uint32_t seq = 0, div = 8;  // (seq 1024: 2% fewer entries, 1.7x the build time on config #4)
    if (const char *e = getenv("KETOGPU_LABEL_SEQ")) seq = (uint32_t)atoi(e);
    if (const char *e = getenv("KETOGPU_LABEL_BATCH_DIV")) div = std::max(1, atoi(e));
    uint32_t r = bits;
    const uint32_t seq_end = (uint32_t)std::min<uint64_t>(n, (uint64_t)bits + seq);
    for (; r < seq_end; r++) {
        search(sr[0], r, 0, true);
        search(sr[0], r, 1, true);
    }
    phase("sequential");
    double t_search = 0, t_merge = 0;
    while (r < n) {
        const uint32_t bs = std::max<uint32_t>((uint32_t)T * 4, r / div);
        const uint32_t e = (uint32_t)std::min<uint64_t>(n, (uint64_t)r + bs);
        const auto tb = Clock::now();
        parallel_chunks(e - r, 8, [&](int tid, uint64_t b, uint64_t f) {
            for (uint64_t k = b; k < f; k++) {
                search(sr[tid], r + (uint32_t)k, 0, false);
                search(sr[tid], r + (uint32_t)k, 1, false);
            }
        });
        t_search += ms_since(tb);
        const auto tm = Clock::now();
        // merge: thread t appends the entries of nodes y with y % T == t (its buckets)
        parallel_chunks((uint64_t)T, 1, [&](int, uint64_t b, uint64_t f) {
            for (uint64_t t = b; t < f; t++)
                for (int d = 0; d < 2; d++)
                    for (auto &x : sr) {
                        for (auto &p : x.add[d][t]) L[d][p.first].push_back(p.second);
                        x.add[d][t].clear();
                    }
        });
        t_merge += ms_since(tm);
        out.batches++;
        r = e;
    }
    if (plog) fprintf(stderr, "[pll] batches: %llu, searches %.1f ms, merges %.1f ms\n",
                      (unsigned long long)out.batches, t_search, t_merge);
    phase("batched");
    for (auto &x : sr) std::vector<uint32_t>().swap(x.vis), std::vector<uint32_t>().swap(x.mark);
    // sorted CSR
    for (int d = 0; d < 2; d++) {
        std::vector<uint64_t> &off = d == 0 ? out.in_off : out.out_off;
        std::vector<uint32_t> &col = d == 0 ? out.in : out.out;
        off.assign((size_t)n + 1, 0);
        for (uint32_t v = 0; v < n; v++) off[v + 1] = off[v] + L[d][v].size();
        col.resize(off[n]);
        parallel_chunks(n, 1 << 14, [&](int, uint64_t b, uint64_t e) {
            for (uint64_t v = b; v < e; v++) {
                std::vector<uint32_t> &l = L[d][v];
                std::sort(l.begin(), l.end());
                std::copy(l.begin(), l.end(), col.begin() + (ptrdiff_t)off[v]);
                std::vector<uint32_t>().swap(l);
            }
        });
    }
    phase("csr");
    out.ms = ms_since(t0);
}
}  // namespace

std::shared_ptr<const ReachLabels> reach_labels_of(const Snapshot &s) {
    // (callers hold the snapshot's shared lock: the version cannot change during the build)
    std::promise<std::shared_ptr<const ReachLabels>> mine;
    std::shared_future<std::shared_ptr<const ReachLabels>> wait;
    {
        std::lock_guard<std::mutex> lk(s.derived_mu);
        if (s.reach_cache && s.reach_cache->version == s.version) return s.reach_cache;
        if (s.reach_building.valid() && s.reach_building_version == s.version) {
            wait = s.reach_building;  // another engine builds this version: wait for it
        } else {
            s.reach_building = mine.get_future().share();
            s.reach_building_version = s.version;
        }
    }
    if (wait.valid()) return wait.get();  // (rethrows the builder's error)
    try {
        auto R = std::make_shared<ReachLabels>();
        build_reach_labels(s, *R);  // outside derived_mu
        R->version = s.version;
        std::shared_ptr<const ReachLabels> done = std::move(R);
        {
            std::lock_guard<std::mutex> lk(s.derived_mu);
            s.reach_cache = done;
            s.reach_building = {};
            s.reach_building_version = ~0ull;
        }
        mine.set_value(done);
        return done;
    } catch (...) {
        {
            std::lock_guard<std::mutex> lk(s.derived_mu);
            s.reach_building = {};
            s.reach_building_version = ~0ull;
        }
        mine.set_exception(std::current_exception());
        throw;
    }
}

namespace {

struct Lists {
    const Snapshot &s;
    const ReachLabels &R;
    // S(x): Lin of the interior entries of rev(x) + its other entries (raw node ids)
    void s_list(uint64_t x, std::vector<uint32_t> &out, uint64_t &mask) const {
        out.clear();
        mask = 0;
        const uint32_t *b = s.rev_col.data() + s.rev_off[x], *e = s.rev_col.data() + s.rev_off[x + 1];
        for (const uint32_t *p = b; p < e; p++) {
            const uint32_t v = *p;
            if (s.writable && (v == s.Dbi || v == s.Dbo)) continue;  // a free slot
            if (v < R.n) {
                mask |= R.min[v];
                out.insert(out.end(), R.in.begin() + (ptrdiff_t)R.in_off[v], R.in.begin() + (ptrdiff_t)R.in_off[v + 1]);
            } else {
                out.push_back(v);
            }
        }
        std::sort(out.begin(), out.end());
        out.erase(std::unique(out.begin(), out.end()), out.end());
    }
    // P(r): Lout(r) for an interior r, else Lout of every entry of fint(r) (the one-edge
    // case r in rev(t) is the raw test against S(t), labels.hpp)
    void p_list(uint64_t r, std::vector<uint32_t> &out, uint64_t &mask) const {
        out.clear();
        if (r < R.n) {
            mask = R.mout[r];
            out.assign(R.out.begin() + (ptrdiff_t)R.out_off[r], R.out.begin() + (ptrdiff_t)R.out_off[r + 1]);
            return;
        }
        mask = 0;
        const uint32_t *b = s.fint_col.data() + s.fint_off[r], *e = s.fint_col.data() + s.fint_off[r + 1];
        for (const uint32_t *p = b; p < e; p++) {
            if (s.writable && *p == s.Df) continue;  // a free slot
            mask |= R.mout[*p];
            out.insert(out.end(), R.out.begin() + (ptrdiff_t)R.out_off[*p], R.out.begin() + (ptrdiff_t)R.out_off[*p + 1]);
        }
        std::sort(out.begin(), out.end());
        out.erase(std::unique(out.begin(), out.end()), out.end());
    }
};

uint32_t pick_head_of(const std::vector<uint32_t> &cnt) {
    uint64_t ne = 0, fit[4] = {0, 0, 0, 0};
    for (uint32_t c : cnt) {
        if (!c) continue;
        ne++;
        for (int k = 0; k < 4; k++) fit[k] += c <= (8u << k) - kHeadFixed;
    }
    return ketogpu::pick_head(ne, fit);
}

}  // namespace

uint32_t pick_head(uint64_t nonempty, const uint64_t fit[4]) {
    if ((fit[3] - fit[2]) * 10 >= nonempty) return 64;
    for (int k = 0; k < 2; k++)
        if (fit[k] * 1000 >= fit[2] * 999) return 8u << k;
    return 32;
}

uint64_t label_s_nodes(const Snapshot &s) { return s.writable ? s.n_cap : s.N; }

bool label_nolabel(uint64_t x, uint32_t permille) {
    return permille && mix64(x * 0x9E3779B97F4A7C15ull + 17) % 1000 < permille;
}

void label_list(const Snapshot &s, const ReachLabels &R, bool p_side, uint64_t x, std::vector<uint32_t> &out,
                uint64_t &mask) {
    const Lists l{s, R};
    if (p_side)
        l.p_list(x, out, mask);
    else
        l.s_list(x, out, mask);
}

void build_labels(const Snapshot &s, uint32_t hs, uint32_t hp, uint32_t rest_permille, uint64_t max_bytes,
                  LabelIndex &out) {
    const auto t0 = Clock::now();
    for (uint32_t h : {hs, hp})
        if (h && h != 8 && h != 16 && h != 32 && h != 64)
            throw Error(KETOGPU_EINVAL, "plan label: heads of 8, 16, 32 or 64 words");
    out = LabelIndex{};
    ReachLabels R;
    build_reach_labels(s, R);
    out.pll_ms = R.ms;
    out.label_entries = R.in.size() + R.out.size();
    const Lists lists{s, R};
    const uint64_t ns = label_s_nodes(s), np = s.Nx;
    out.s_nodes = ns;
    out.p_nodes = np;
    // pass 1: list lengths
    std::vector<uint32_t> cs(ns), cp(np);
    const int T = build_threads();
    std::vector<std::vector<uint32_t>> tmp(T);
    parallel_chunks(ns, 1 << 14, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t m;
        for (uint64_t x = b; x < e; x++) {
            lists.s_list(x, tmp[tid], m);
            cs[x] = (uint32_t)tmp[tid].size();
        }
    });
    parallel_chunks(np, 1 << 14, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t m;
        for (uint64_t x = b; x < e; x++) {
            lists.p_list(x, tmp[tid], m);
            cp[x] = (uint32_t)tmp[tid].size();
        }
    });
    out.hs = hs ? hs : pick_head_of(cs);
    out.hp = hp ? hp : pick_head_of(cp);
    // overflow lists (whole, 16-word aligned) after the heads
    auto layout = [](const std::vector<uint32_t> &cnt, uint32_t h, std::vector<uint64_t> &ovf, uint64_t &lists) {
        ovf.resize(cnt.size());
        uint64_t acc = (uint64_t)cnt.size() * h;  // a multiple of 8 words
        acc = (acc + 15) / 16 * 16;
        lists = 0;
        for (size_t x = 0; x < cnt.size(); x++) {
            ovf[x] = 0;
            if (cnt[x] > h - kHeadFixed) {
                ovf[x] = acc;
                acc += ((uint64_t)cnt[x] + 15) / 16 * 16;
                lists++;
            }
        }
        return acc;
    };
    std::vector<uint64_t> os, op;
    const uint64_t ws = layout(cs, out.hs, os, out.s_overflow), wp = layout(cp, out.hp, op, out.p_overflow);
    if (ws / 16 >= (1ull << 32) || wp / 16 >= (1ull << 32))
        throw Error(KETOGPU_EINVAL, "plan label: head arrays pass 2^36 words");
    if (max_bytes && 4 * (ws + wp) > max_bytes)
        throw Error(KETOGPU_ENOMEM, "plan label: " + std::to_string(4 * (ws + wp)) + " bytes of labels, budget " +
                                        std::to_string(max_bytes));
    out.S.assign(ws, 0xFFFFFFFFu);
    out.P.assign(wp, 0xFFFFFFFFu);
    // pass 2: heads and overflow lists
    auto write = [&](std::vector<uint32_t> &A, uint32_t h, const std::vector<uint64_t> &ovf, uint64_t x,
                     const std::vector<uint32_t> &l, uint64_t mask, bool nolabel) {
        uint32_t *hd = A.data() + x * h;
        hd[0] = nolabel ? kNoLabel : (uint32_t)l.size();
        hd[1] = (uint32_t)(ovf[x] / 16);
        hd[2] = (uint32_t)mask;
        hd[3] = (uint32_t)(mask >> 32);
        // an overflowing list lies whole in the overflow region, its first h - 4 entries also
        // in the head (most hits are found there without the second read)
        const size_t inl = std::min<size_t>(l.size(), h - kHeadFixed);
        std::copy(l.begin(), l.begin() + (ptrdiff_t)inl, hd + kHeadFixed);
        if (l.size() > h - kHeadFixed) std::copy(l.begin(), l.end(), A.data() + ovf[x]);
    };
    std::atomic<uint64_t> es{0}, ep{0}, nl{0};
    parallel_chunks(ns, 1 << 14, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t m, en = 0, nn = 0;
        for (uint64_t x = b; x < e; x++) {
            lists.s_list(x, tmp[tid], m);
            const bool nolabel = cs[x] && label_nolabel(x, rest_permille);
            write(out.S, out.hs, os, x, tmp[tid], m, nolabel);
            en += tmp[tid].size();
            nn += nolabel;
        }
        es += en;
        nl += nn;
    });
    parallel_chunks(np, 1 << 14, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t m, en = 0;
        for (uint64_t x = b; x < e; x++) {
            lists.p_list(x, tmp[tid], m);
            write(out.P, out.hp, op, x, tmp[tid], m, false);
            en += tmp[tid].size();
        }
        ep += en;
    });
    out.s_entries = es;
    out.p_entries = ep;
    out.s_nolabel = nl;
    out.build_ms = ms_since(t0);
}

}  // namespace ketogpu

// ------------------------------------------------------------------ C ABI (tools, tests)
struct ketogpu_label_index {
    ketogpu::LabelIndex li;
};

extern "C" {

int ketogpu_label_index_build(const ketogpu_snapshot *s, uint32_t s_head_words, uint32_t p_head_words,
                              ketogpu_label_index **out) {
    try {
        if (!s || !out) throw ketogpu::Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        const auto *snap = reinterpret_cast<const ketogpu::Snapshot *>(s);
        std::shared_lock<std::shared_mutex> lk(snap->mu);
        auto l = std::make_unique<ketogpu_label_index>();
        ketogpu::build_labels(*snap, s_head_words, p_head_words, 0, 0, l->li);
        *out = l.release();
    } catch (const ketogpu::Error &e) {
        ketogpu::set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        ketogpu::set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

int ketogpu_label_index_view(const ketogpu_label_index *l, ketogpu_label_view *out) {
    if (!l || !out) {
        ketogpu::set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const ketogpu::LabelIndex &li = l->li;
    out->s_head_words = li.hs;
    out->p_head_words = li.hp;
    out->s_words = li.S.data();
    out->p_words = li.P.data();
    out->num_s_words = li.S.size();
    out->num_p_words = li.P.size();
    out->s_nodes = li.s_nodes;
    out->p_nodes = li.p_nodes;
    out->s_entries = li.s_entries;
    out->p_entries = li.p_entries;
    out->s_overflow = li.s_overflow;
    out->p_overflow = li.p_overflow;
    out->label_entries = li.label_entries;
    out->pll_ms = li.pll_ms;
    out->build_ms = li.build_ms;
    return KETOGPU_OK;
}

void ketogpu_label_index_free(ketogpu_label_index *l) { delete l; }

}  // extern "C"
