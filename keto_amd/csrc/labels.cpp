// labels.cpp — builds the closure labels of plan "label" (labels.hpp).
#include "labels.hpp"

#include <algorithm>
#include <chrono>
#include <memory>
#include <random>
#include <shared_mutex>

namespace ketogpu {

namespace {

constexpr uint32_t kRawMax = 4096;  // a label's entries before deduplication: beyond, no label

struct Ctx {
    const Snapshot &s;
    const CoreIndex &ci;
    int mode;
    uint32_t words;  // S block words: a label holds at most words - 1 nodes
    // the S list of node x (mode B: x = t, S = rev(t) + closures of its interior entries;
    // mode F: x = r, S = {r} + fint(r) + closures of its entries); false: no label
    bool label(uint64_t x, std::vector<uint32_t> &out) const {
        out.clear();
        const int d = mode == 0 ? 1 : 0;  // the closures' direction: backward for B, forward for F
        const uint64_t *off = mode == 0 ? s.rev_off.data() : s.fint_off.data();
        const uint32_t *col = mode == 0 ? s.rev_col.data() : s.fint_col.data();
        const uint32_t *b = col + off[x], *e = col + off[x + 1];
        if (mode == 1) out.push_back((uint32_t)x);
        for (const uint32_t *p = b; p < e; p++) {
            out.push_back(*p);
            if (*p >= s.Ni) continue;  // mode B: a source entry (only r itself can be it)
            const uint32_t n = ci.clo_len[d][*p];
            if (n == NONE) return false;
            if (out.size() + n > kRawMax) return false;
            const CoreRec *c = ci.rec[d].data() + ci.clo_beg[d][*p];
            for (uint32_t k = 0; k < n; k++) out.push_back(c[k].node);
        }
        std::sort(out.begin(), out.end());
        out.erase(std::unique(out.begin(), out.end()), out.end());
        return out.size() < words;
    }
    uint64_t s_nodes() const { return mode == 0 ? s.N : s.Nx; }
    bool nonempty(uint64_t x) const {
        const uint64_t *off = mode == 0 ? s.rev_off.data() : s.fint_off.data();
        return off[x + 1] > off[x];
    }
};

// labelled share of a sample of S nodes with a non-empty row
double sample_coverage(const Ctx &c, uint64_t sample) {
    const uint64_t n = c.s_nodes();
    if (!n) return 0;
    std::vector<uint64_t> pick;
    std::mt19937_64 rng(0x4B45544Full);
    for (uint64_t k = 0; k < 4 * sample && pick.size() < sample; k++) {
        const uint64_t x = rng() % n;
        if (c.nonempty(x)) pick.push_back(x);
    }
    if (pick.empty()) return 1.0;
    std::atomic<uint64_t> hit{0};
    std::vector<std::vector<uint32_t>> tmp(build_threads());
    parallel_chunks(pick.size(), 256, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t h = 0;
        for (uint64_t i = b; i < e; i++) h += c.label(pick[i], tmp[tid]);
        hit += h;
    });
    return (double)hit.load() / (double)pick.size();
}

}  // namespace

void build_labels(const Snapshot &s, const CoreIndex &ci, int mode, double min_coverage, LabelIndex &out,
                  uint32_t s_words) {
    if (s_words != 64 && s_words != 128) throw Error(KETOGPU_EINVAL, "plan label: S blocks of 64 or 128 words");
    const auto t0 = std::chrono::steady_clock::now();
    out = LabelIndex{};
    out.s_words = s_words;
    for (int m = 0; m < 2; m++)
        if (ci.clo_len[m == 0 ? 1 : 0].size() == s.Ni) out.coverage[m] = sample_coverage(Ctx{s, ci, m, s_words}, 20000);
    if (mode < 0) {
        mode = out.coverage[0] >= out.coverage[1] ? 0 : 1;
        if (out.coverage[mode] < min_coverage) {
            out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            return;
        }
    }
    if (ci.clo_len[mode == 0 ? 1 : 0].size() != s.Ni)
        throw Error(KETOGPU_EINVAL, "plan label: the core index has no closure rows in that direction");
    const Ctx c{s, ci, mode, s_words};
    out.mode = mode;
    // S blocks
    const uint64_t ns = c.s_nodes();
    out.s_nodes = ns;
    out.S.assign(ns * s_words, 0xFFFFFFFFu);
    std::atomic<uint64_t> covered{0}, nonempty{0};
    std::vector<std::vector<uint32_t>> tmp(build_threads());
    parallel_chunks(ns, 1 << 14, [&](int tid, uint64_t b, uint64_t e) {
        uint64_t cv = 0, ne = 0;
        for (uint64_t x = b; x < e; x++) {
            uint32_t *blk = out.S.data() + x * s_words;
            const bool has = c.nonempty(x);
            ne += has;
            if (!c.label(x, tmp[tid])) continue;  // count stays 0xFFFFFFFF: no label
            cv += has;
            blk[0] = (uint32_t)tmp[tid].size();
            std::copy(tmp[tid].begin(), tmp[tid].end(), blk + 1);
        }
        covered += cv;
        nonempty += ne;
    });
    out.covered = covered;
    out.nonempty = nonempty;
    // P blocks: mode B {r} + fint(r) for every expandable r, mode F rev(t) for every node t
    const uint64_t np = mode == 0 ? s.Nx : s.N;
    const uint64_t *off = mode == 0 ? s.fint_off.data() : s.rev_off.data();
    const uint32_t *col = mode == 0 ? s.fint_col.data() : s.rev_col.data();
    const uint64_t extra = mode == 0 ? 1 : 0;  // r itself
    auto plen = [&](uint64_t x) { return off[x + 1] - off[x] + extra; };
    {  // the smallest block whose inline entries hold >= 95% of the non-empty rows
        uint64_t fit[3] = {0, 0, 0}, ne = 0;
        for (uint64_t x = 0; x < np; x++) {
            const uint64_t n = plen(x);
            if (!n) continue;
            ne++;
            for (int k = 0; k < 3; k++) fit[k] += n <= (16u << k) - 2;
        }
        out.pb = 64;
        for (int k = 0; k < 3; k++)
            if (fit[k] * 20 >= ne * 19) {
                out.pb = 16u << k;
                break;
            }
    }
    const uint32_t pb = out.pb, inl = pb - 2;
    out.p_nodes = np;
    std::vector<uint64_t> ovf(np, 0);
    uint64_t acc = 0;
    for (uint64_t x = 0; x < np; x++) {
        ovf[x] = acc;
        const uint64_t n = plen(x);
        if (n > inl) acc += (n - inl + 15) / 16 * 16;  // 16-word aligned
    }
    const uint64_t obase = np * pb;  // a multiple of 16 words
    if ((obase + acc) / 16 >= (1ull << 32)) throw Error(KETOGPU_EINVAL, "plan label: P rows pass 2^36 words");
    out.P.assign(obase + acc, 0xFFFFFFFFu);
    parallel_chunks(np, 1 << 15, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t x = b; x < e; x++) {
            const uint64_t n = plen(x);
            uint32_t *blk = out.P.data() + x * pb;
            uint32_t *ov = out.P.data() + obase + ovf[x];
            blk[0] = (uint32_t)n;
            blk[1] = n > inl ? (uint32_t)((obase + ovf[x]) / 16) : 0u;
            for (uint64_t k = 0; k < n; k++) {
                const uint32_t v = extra && k == 0 ? (uint32_t)x : col[off[x] + k - extra];
                if (k < inl)
                    blk[2 + k] = v;
                else
                    ov[k - inl] = v;
            }
        }
    });
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace ketogpu

// ------------------------------------------------------------------ C ABI (tools, tests)
struct ketogpu_label_index {
    ketogpu::LabelIndex li;
};

extern "C" {

int ketogpu_label_index_build(const ketogpu_snapshot *s, const uint32_t closure_cap[2], int mode, uint32_t s_words,
                              ketogpu_label_index **out) {
    try {
        if (!s || !closure_cap || !out || mode < -1 || mode > 1) throw ketogpu::Error(KETOGPU_EINVAL, "bad argument");
        *out = nullptr;
        const auto *snap = reinterpret_cast<const ketogpu::Snapshot *>(s);
        std::shared_lock<std::shared_mutex> lk(snap->mu);
        ketogpu::CoreIndex ci;
        const uint32_t block[2] = {0, 0};
        ketogpu::build_core_index(*snap, closure_cap, block, ci);
        auto l = std::make_unique<ketogpu_label_index>();
        ketogpu::build_labels(*snap, ci, mode, 0.5, l->li, s_words);
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
    out->mode = li.mode;
    out->s_block_words = li.s_words;
    out->p_block_words = li.pb;
    out->p_words = li.P.data();
    out->s_words = li.S.data();
    out->num_p_words = li.P.size();
    out->num_s_words = li.S.size();
    out->p_nodes = li.p_nodes;
    out->s_nodes = li.s_nodes;
    out->labelled = li.covered;
    out->nonempty = li.nonempty;
    out->coverage_b = li.coverage[0];
    out->coverage_f = li.coverage[1];
    return KETOGPU_OK;
}

void ketogpu_label_index_free(ketogpu_label_index *l) { delete l; }

}  // extern "C"
