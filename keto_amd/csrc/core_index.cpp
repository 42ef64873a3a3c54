// core_index.cpp — builds plan "core"'s record arrays and closure rows (core_index.hpp).
#include "core_index.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>

namespace ketogpu {

int build_threads() {
    if (const char *e = getenv("KETOGPU_BUILD_THREADS")) return std::max(1, atoi(e));
    // the GPU box's job quota is 16 cores (nproc shows the whole machine)
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

namespace {

// interior adjacency of one direction: forward fint(v) (interior successors), backward the
// interior predecessors (the prefix of the sorted rev(v) below Ni)
struct Adj {
    const uint32_t *col;
    std::vector<uint64_t> beg;
    std::vector<uint32_t> deg;
    const uint32_t *row(uint32_t v, uint32_t &n) const {
        n = deg[v];
        return col + beg[v];
    }
};

// a bounded breadth-first closure with a small open-addressing visited set (stamped, so
// it is never cleared)
struct Closer {
    static constexpr uint32_t kSlots = 1024;  // > 2 * (cap + 1) for every cap we accept
    uint32_t key[kSlots], stamp[kSlots] = {0};
    uint32_t gen = 0;
    std::vector<uint32_t> queue;
    bool insert(uint32_t u) {
        uint32_t h = (u * 2654435761u) >> 22;  // 10 bits
        for (;; h = (h + 1) & (kSlots - 1)) {
            if (stamp[h] != gen) {
                stamp[h] = gen;
                key[h] = u;
                return true;
            }
            if (key[h] == u) return false;
        }
    }
    // Desc+(v) / Anc+(v) without v itself into out (sorted); false when it has more than
    // cap nodes (or reaches a node known to overflow: its closure is contained in v's)
    bool run(const Adj &a, uint32_t v, uint32_t cap, const std::vector<std::atomic<uint8_t>> &over,
             std::vector<uint32_t> &out) {
        out.clear();
        uint32_t n0;
        a.row(v, n0);
        if (n0 > cap) return false;
        if (++gen == 0) {  // stamps wrapped: clear once
            std::fill(stamp, stamp + kSlots, 0u);
            gen = 1;
        }
        insert(v);
        queue.assign(1, v);
        for (size_t head = 0; head < queue.size(); head++) {
            uint32_t n;
            const uint32_t *r = a.row(queue[head], n);
            for (uint32_t k = 0; k < n; k++) {
                const uint32_t y = r[k];
                if (over[y].load(std::memory_order_relaxed)) return false;
                if (!insert(y)) continue;
                out.push_back(y);
                if (out.size() > cap) return false;
                queue.push_back(y);
            }
        }
        std::sort(out.begin(), out.end());
        return true;
    }
};

}  // namespace

void build_core_index(const Snapshot &s, const uint32_t cap_in[2], const uint32_t block_in[2], CoreIndex &out,
                      uint64_t max_bytes) {
    uint64_t bytes_before = 0;  // records of the directions already laid out
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t Ni = s.Ni;
    if (s.writable) throw Error(KETOGPU_EINVAL, "plan core: writable snapshots change closures in place");
    Adj adj[2];
    adj[0].col = s.fint_col.data();
    adj[1].col = s.rev_col.data();
    for (int d = 0; d < 2; d++) {
        adj[d].beg.resize(Ni);
        adj[d].deg.resize(Ni);
    }
    parallel_chunks(Ni, 1 << 16, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t v = b; v < e; v++) {
            adj[0].beg[v] = s.fint_off[v];
            adj[0].deg[v] = (uint32_t)(s.fint_off[v + 1] - s.fint_off[v]);
            const uint32_t *rb = s.rev_col.data() + s.rev_off[v], *re = s.rev_col.data() + s.rev_off[v + 1];
            adj[1].beg[v] = s.rev_off[v];
            adj[1].deg[v] = (uint32_t)(std::lower_bound(rb, re, Ni) - rb);
        }
    });
    for (int d = 0; d < 2; d++) {
        const uint32_t cap = std::min<uint32_t>(cap_in[d], Closer::kSlots / 2 - 2);
        // closures: per node its length (NONE: no closure row) and the thread-local
        // buffer it sits in
        std::vector<uint32_t> clen(Ni, NONE);
        std::vector<std::pair<uint32_t, uint64_t>> where(cap ? Ni : 0);  // (thread, offset)
        const int T = build_threads();
        std::vector<std::vector<uint32_t>> buf(T);
        if (cap) {
            std::vector<std::atomic<uint8_t>> over(Ni);
            for (auto &x : over) x.store(0, std::memory_order_relaxed);
            std::vector<Closer> cl(T);
            std::vector<std::vector<uint32_t>> tmp(T);
            parallel_chunks(Ni, 1 << 12, [&](int tid, uint64_t b, uint64_t e) {
                for (uint64_t v = b; v < e; v++) {
                    if (!cl[tid].run(adj[d], (uint32_t)v, cap, over, tmp[tid])) {
                        over[v].store(1, std::memory_order_relaxed);
                        continue;
                    }
                    clen[v] = (uint32_t)tmp[tid].size();
                    where[v] = {(uint32_t)tid, buf[tid].size()};
                    buf[tid].insert(buf[tid].end(), tmp[tid].begin(), tmp[tid].end());
                }
            });
        }
        // layout: core rows, closure rows, node blocks, overflow rows
        std::vector<uint32_t> cbeg(Ni), kbeg(Ni, 0);
        uint64_t pos = 0;
        for (uint32_t v = 0; v < Ni; v++) {
            cbeg[v] = (uint32_t)pos;
            pos += adj[d].deg[v];
            if (pos >= (1ull << 32)) throw Error(KETOGPU_EINVAL, "plan core: core rows pass 2^32 records");
        }
        uint64_t nclo = 0, eclo = 0;
        for (uint32_t v = 0; v < Ni; v++)
            if (clen[v] != NONE) {
                kbeg[v] = (uint32_t)pos;
                pos += clen[v];
                nclo++;
                eclo += clen[v];
                if (pos >= (1ull << 32)) throw Error(KETOGPU_EINVAL, "plan core: closure rows pass 2^32 records");
            }
        auto rec_of = [&](uint32_t u) -> CoreRec {
            if (u >= Ni) return CoreRec{u, 0, 0, 0};
            if (clen[u] != NONE && clen[u]) return CoreRec{u, clen[u], kbeg[u], kRecClosure};
            return CoreRec{u, adj[d].deg[u], cbeg[u], 0};
        };
        // node blocks of the seed rows: forward fint(v) of every expandable v, backward
        // rev(v) of every node
        const uint64_t nodes = d == 0 ? s.Nx : s.N;
        const uint64_t *off = d == 0 ? s.fint_off.data() : s.rev_off.data();
        const uint32_t *col = d == 0 ? s.fint_col.data() : s.rev_col.data();
        uint32_t blk = block_in[d];
        if (!blk) {  // the smallest block holding >= 95% of the non-empty rows
            std::vector<uint64_t> hist(6, 0);  // rows of <= 3, 7, 15, 31 entries, longer, empty
            for (uint64_t v = 0; v < nodes; v++) {
                const uint64_t n = off[v + 1] - off[v];
                hist[!n ? 5 : n <= 3 ? 0 : n <= 7 ? 1 : n <= 15 ? 2 : n <= 31 ? 3 : 4]++;
            }
            const uint64_t nonempty = nodes - hist[5];
            uint64_t acc = 0;
            blk = 32;
            for (int k = 0; k < 4; k++) {
                acc += hist[k];
                if (acc * 20 >= nonempty * 19) {
                    blk = 4u << k;
                    break;
                }
            }
        }
        if (blk < 4 || blk > 32 || (blk & (blk - 1))) throw Error(KETOGPU_EINVAL, "plan core: block of 4, 8, 16 or 32 records");
        uint32_t lg = 0;
        while ((1u << lg) < blk) lg++;
        const uint64_t bbase = (pos + blk - 1) / blk * blk;  // blocks aligned to their size
        std::vector<uint64_t> ovf(nodes, 0);  // overflow row starts (exclusive scan of the long rows)
        uint64_t nover = 0, acc = 0;
        for (uint64_t v = 0; v < nodes; v++) {
            const uint64_t n = off[v + 1] - off[v];
            ovf[v] = acc;
            if (n >= blk) acc += n, nover++;
        }
        const uint64_t obase = bbase + (nodes << lg);
        const uint64_t total = obase + acc;
        if (max_bytes && (bytes_before + total) * sizeof(CoreRec) > max_bytes)
            throw Error(KETOGPU_ENOMEM, "plan core: " + std::to_string((bytes_before + total) * sizeof(CoreRec)) +
                                            " bytes of records, budget " + std::to_string(max_bytes));
        bytes_before += total;
        std::vector<CoreRec> &R = out.rec[d];
        R.clear();
        R.resize(total);
        parallel_chunks(Ni, 1 << 14, [&](int, uint64_t b, uint64_t e) {
            for (uint64_t v = b; v < e; v++) {
                uint32_t n;
                const uint32_t *row = adj[d].row((uint32_t)v, n);
                for (uint32_t k = 0; k < n; k++) R[cbeg[v] + k] = rec_of(row[k]);
                if (clen[v] != NONE) {
                    const uint32_t *c = buf[where[v].first].data() + where[v].second;
                    for (uint32_t k = 0; k < clen[v]; k++) R[kbeg[v] + k] = CoreRec{c[k], 0, 0, kRecTerminal};
                }
            }
        });
        parallel_chunks(nodes, 1 << 16, [&](int, uint64_t b, uint64_t e) {
            for (uint64_t v = b; v < e; v++) {
                const uint64_t n = off[v + 1] - off[v];
                CoreRec *bl = R.data() + bbase + (v << lg);
                const uint64_t first = n < blk ? bbase + (v << lg) + 1 : obase + ovf[v];
                bl[0] = CoreRec{(uint32_t)n, (uint32_t)first, (uint32_t)(first >> 32), 0};
                for (uint64_t k = 0; k < n; k++) R[first + k] = rec_of(col[off[v] + k]);
                for (uint64_t k = n < blk ? n + 1 : 1; k < blk; k++) bl[k] = CoreRec{NONE, 0, 0, 0};
            }
        });
        out.clo_len[d] = std::move(clen);
        out.clo_beg[d] = std::move(kbeg);
        out.block_base[d] = bbase;
        out.block_log[d] = lg;
        out.overflow_rows[d] = nover;
        out.closure_nodes[d] = nclo;
        out.closure_entries[d] = eclo;
    }
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace ketogpu

// ------------------------------------------------------------------ C ABI (tools, tests)
struct ketogpu_core_index {
    ketogpu::CoreIndex ci;
};

extern "C" {

int ketogpu_core_index_build(const ketogpu_snapshot *s, const uint32_t closure_cap[2], const uint32_t block[2],
                             ketogpu_core_index **out) {
    try {
        if (!s || !closure_cap || !block || !out) throw ketogpu::Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        auto c = std::make_unique<ketogpu_core_index>();
        const auto *snap = reinterpret_cast<const ketogpu::Snapshot *>(s);
        std::shared_lock<std::shared_mutex> lk(snap->mu);
        ketogpu::build_core_index(*snap, closure_cap, block, c->ci);
        *out = c.release();
    } catch (const ketogpu::Error &e) {
        ketogpu::set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        ketogpu::set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

int ketogpu_core_index_view(const ketogpu_core_index *c, int direction, ketogpu_core_records *out) {
    if (!c || !out || direction < 0 || direction > 1) {
        ketogpu::set_last_error("null argument or direction not 0/1");
        return KETOGPU_EINVAL;
    }
    const ketogpu::CoreIndex &ci = c->ci;
    out->records = reinterpret_cast<const uint32_t *>(ci.rec[direction].data());
    out->num_records = ci.rec[direction].size();
    out->block_base = ci.block_base[direction];
    out->block_records = 1u << ci.block_log[direction];
    out->overflow_rows = ci.overflow_rows[direction];
    out->closure_nodes = ci.closure_nodes[direction];
    out->closure_entries = ci.closure_entries[direction];
    return KETOGPU_OK;
}

void ketogpu_core_index_free(ketogpu_core_index *c) { delete c; }

}  // extern "C"
