// synth.cpp — synthetic workloads of BASELINE.json (tooling for bench.py and tests,
// not part of the engine ABI).  Config #2: synthetic RBAC,
//   users u0..u{U-1}; groups g0..g{G-1} in 4 levels (1% / 4% / 15% / 80%), every group
//   below the top has 1-2 parents one level up (groups:gP#member@(groups:gC#member));
//   memberships groups:g#member@u, Poisson(mean) per user into leaf groups chosen by
//   Zipf(s) ; the remaining tuples are grants docs:dK#viewer@(groups:g#member) (80%) or
//   @u (20%) over D docs.  Longest path doc -> g0 -> g1 -> g2 -> g3 -> user = 5 edges.
//   Checks docs:d#viewer@u: 50% constructed positives (a sampled grant path), 50%
//   uniform random pairs.
// Rows are emitted already in the reference's ORDER BY order under SQLite semantics
// (namespace id, then BINARY object, relation, NULL subject_id first, ...), i.e. what
// the snapshot loader reads from the database.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

namespace {

struct Rng {  // splitmix64
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
    double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

// ranks of 0..n-1 in the lexicographic order of their decimal strings
std::vector<uint32_t> lex_order(uint64_t n) {
    std::vector<uint32_t> order;
    order.reserve(n);
    if (!n) return order;
    order.push_back(0);
    std::vector<uint64_t> st;
    for (int d = 9; d >= 1; d--)
        if ((uint64_t)d < n) st.push_back(d);
    while (!st.empty()) {
        uint64_t v = st.back();
        st.pop_back();
        order.push_back((uint32_t)v);
        for (int e = 9; e >= 0; e--) {
            uint64_t c = v * 10 + e;
            if (c < n) st.push_back(c);
        }
    }
    return order;
}

struct Col {
    std::vector<char> data;
    std::vector<uint64_t> off{0};
    void put(const char *p, size_t n) {
        data.insert(data.end(), p, p + n);
        off.push_back(data.size());
    }
    void put_num(char prefix, uint64_t v) {
        char b[24];
        int n = snprintf(b, sizeof b, "%c%llu", prefix, (unsigned long long)v);
        put(b, (size_t)n);
    }
    void empty() { off.push_back(data.size()); }
};

}  // namespace

struct ks_rbac {
    // rows (columnar, ketogpu_row_batch layout)
    std::vector<int32_t> ns, ss_ns;
    std::vector<uint8_t> kind;
    Col obj, rel, sid, ss_obj, ss_rel;
    // checks: doc index, user index, constructed-positive flag
    std::vector<uint32_t> chk_doc, chk_user;
    std::vector<uint8_t> chk_pos;
    // request columns for the checks
    Col rq_ns, rq_obj, rq_rel, rq_sid;
    uint64_t n_parent = 0, n_member = 0, n_grant = 0;
};

extern "C" {

typedef struct {
    uint64_t users, groups, docs, tuples, checks, seed;
    double zipf_s, member_mean;
    uint64_t check_seed; /* 0: checks continue the graph's random stream */
} ks_rbac_params;

typedef struct {
    uint64_t n;
    const int32_t *namespace_id;
    const char *object_data;
    const uint64_t *object_off;
    const char *relation_data;
    const uint64_t *relation_off;
    const uint8_t *subject_kind;
    const char *subject_id_data;
    const uint64_t *subject_id_off;
    const int32_t *ss_namespace_id;
    const char *ss_object_data;
    const uint64_t *ss_object_off;
    const char *ss_relation_data;
    const uint64_t *ss_relation_off;
    // checks
    uint64_t n_checks;
    const uint32_t *chk_doc, *chk_user;
    const uint8_t *chk_pos;
    const char *rq_ns_data;
    const uint64_t *rq_ns_off;
    const char *rq_obj_data;
    const uint64_t *rq_obj_off;
    const char *rq_rel_data;
    const uint64_t *rq_rel_off;
    const char *rq_sid_data;
    const uint64_t *rq_sid_off;
    uint64_t n_parent, n_member, n_grant;
} ks_rbac_view;

ks_rbac *ks_rbac_generate(const ks_rbac_params *p) {
    auto *w = new ks_rbac();
    Rng rng(p->seed);
    const uint64_t U = p->users, G = p->groups, D = p->docs;
    // ---- group levels
    uint64_t lv[4];
    lv[0] = std::max<uint64_t>(1, G / 100);
    lv[1] = std::max<uint64_t>(1, G * 4 / 100);
    lv[2] = std::max<uint64_t>(1, G * 15 / 100);
    lv[3] = G - lv[0] - lv[1] - lv[2];
    uint64_t base[5] = {0, lv[0], lv[0] + lv[1], lv[0] + lv[1] + lv[2], G};
    // children[g] = child groups of g (edge g -> child)
    std::vector<std::vector<uint32_t>> children(G);
    for (int l = 1; l < 4; l++)
        for (uint64_t c = base[l]; c < base[l + 1]; c++) {
            int np = 1 + (int)rng.below(2);
            uint32_t p0 = (uint32_t)(base[l - 1] + rng.below(lv[l - 1]));
            children[p0].push_back((uint32_t)c);
            if (np == 2 && lv[l - 1] > 1) {
                uint32_t p1;
                do p1 = (uint32_t)(base[l - 1] + rng.below(lv[l - 1]));
                while (p1 == p0);
                children[p1].push_back((uint32_t)c);
            }
            w->n_parent += np == 2 && lv[l - 1] > 1 ? 2 : 1;
        }
    // ---- memberships: Poisson(mean) per user into leaf groups by Zipf(s)
    const uint64_t L = lv[3];
    std::vector<double> cdf(L);
    {
        double acc = 0;
        for (uint64_t k = 0; k < L; k++) acc += 1.0 / std::pow((double)(k + 1), p->zipf_s), cdf[k] = acc;
        for (auto &x : cdf) x /= acc;
    }
    // leaf rank k -> leaf group id (a fixed random permutation so hubs are spread)
    std::vector<uint32_t> leaf_perm(L);
    std::iota(leaf_perm.begin(), leaf_perm.end(), (uint32_t)base[3]);
    for (uint64_t i = L; i > 1; i--) std::swap(leaf_perm[i - 1], leaf_perm[rng.below(i)]);
    std::vector<std::vector<uint32_t>> members(G);
    std::poisson_distribution<int> pois(p->member_mean);
    std::mt19937_64 mt(p->seed ^ 0x5bd1e995);
    for (uint64_t u = 0; u < U; u++) {
        int k = pois(mt);
        for (int j = 0; j < k; j++) {
            uint64_t r = std::lower_bound(cdf.begin(), cdf.end(), rng.unit()) - cdf.begin();
            if (r >= L) r = L - 1;
            members[leaf_perm[r]].push_back((uint32_t)u);
            w->n_member++;
        }
    }
    // ---- grants fill the tuple budget
    uint64_t used = w->n_parent + w->n_member;
    uint64_t n_grant = p->tuples > used ? p->tuples - used : D;
    std::vector<std::vector<uint32_t>> doc_groups(D), doc_users(D);
    for (uint64_t i = 0; i < n_grant; i++) {
        uint64_t d = rng.below(D);
        if (rng.unit() < 0.8)
            doc_groups[d].push_back((uint32_t)rng.below(G));
        else
            doc_users[d].push_back((uint32_t)rng.below(U));
    }
    w->n_grant = n_grant;
    // ---- emit rows in ORDER BY order (SQLite: BINARY strings, NULL subject_id first)
    std::vector<uint32_t> urank(U), grank(G);
    {
        auto o = lex_order(U);
        for (uint64_t i = 0; i < U; i++) urank[o[i]] = (uint32_t)i;
        auto og = lex_order(G);
        for (uint64_t i = 0; i < G; i++) grank[og[i]] = (uint32_t)i;
    }
    auto by_u = [&](uint32_t a, uint32_t b) { return urank[a] < urank[b]; };
    auto by_g = [&](uint32_t a, uint32_t b) { return grank[a] < grank[b]; };
    uint64_t total = w->n_parent + w->n_member + n_grant;
    w->ns.reserve(total);
    w->kind.reserve(total);
    w->ss_ns.reserve(total);
    auto row_set = [&](int32_t ns, char op, uint64_t o, const char *rel, char sp, uint64_t so, int32_t sns,
                       const char *srel) {
        w->ns.push_back(ns);
        w->kind.push_back(1);
        w->ss_ns.push_back(sns);
        w->obj.put_num(op, o);
        w->rel.put(rel, strlen(rel));
        w->sid.empty();
        w->ss_obj.put_num(sp, so);
        w->ss_rel.put(srel, strlen(srel));
    };
    auto row_id = [&](int32_t ns, char op, uint64_t o, const char *rel, uint64_t u) {
        w->ns.push_back(ns);
        w->kind.push_back(0);
        w->ss_ns.push_back(0);
        w->obj.put_num(op, o);
        w->rel.put(rel, strlen(rel));
        w->sid.put_num('u', u);
        w->ss_obj.empty();
        w->ss_rel.empty();
    };
    // namespace 1: groups (ordered by object string)
    for (uint32_t g : lex_order(G)) {
        auto &ch = children[g];
        std::sort(ch.begin(), ch.end(), by_g);
        for (uint32_t c : ch) row_set(1, 'g', g, "member", 'g', c, 1, "member");
        auto &m = members[g];
        std::sort(m.begin(), m.end(), by_u);
        for (uint32_t u : m) row_id(1, 'g', g, "member", u);
    }
    // namespace 2: docs
    for (uint32_t d : lex_order(D)) {
        auto &dg = doc_groups[d];
        std::sort(dg.begin(), dg.end(), by_g);
        for (uint32_t g : dg) row_set(2, 'd', d, "viewer", 'g', g, 1, "member");
        auto &du = doc_users[d];
        std::sort(du.begin(), du.end(), by_u);
        for (uint32_t u : du) row_id(2, 'd', d, "viewer", u);
    }
    // ---- checks
    if (p->check_seed) rng = Rng(p->check_seed);
    const uint64_t C = p->checks;
    w->chk_doc.resize(C);
    w->chk_user.resize(C);
    w->chk_pos.resize(C);
    for (uint64_t i = 0; i < C; i++) {
        uint64_t d = rng.below(D);
        uint64_t u = rng.below(U);
        bool pos = false;
        if (rng.unit() < 0.5) {
            // constructed positive: sample a grant path from a doc that has grants
            for (int tries = 0; tries < 64 && !pos; tries++) {
                uint64_t dd = rng.below(D);
                uint64_t ng = doc_groups[dd].size(), nu = doc_users[dd].size();
                if (!ng && !nu) continue;
                uint64_t pick = rng.below(ng + nu);
                if (pick >= ng) {
                    d = dd, u = doc_users[dd][pick - ng], pos = true;
                    break;
                }
                uint32_t g = doc_groups[dd][pick];
                for (int hop = 0; hop < 8; hop++) {  // walk down to a member
                    uint64_t nc = children[g].size(), nm = members[g].size();
                    if (!nc && !nm) break;
                    uint64_t k = rng.below(nc + nm);
                    if (k >= nc) {
                        d = dd, u = members[g][k - nc], pos = true;
                        break;
                    }
                    g = children[g][k];
                }
            }
        }
        w->chk_doc[i] = (uint32_t)d;
        w->chk_user[i] = (uint32_t)u;
        w->chk_pos[i] = pos;
        w->rq_ns.put("docs", 4);
        w->rq_obj.put_num('d', d);
        w->rq_rel.put("viewer", 6);
        w->rq_sid.put_num('u', u);
    }
    return w;
}

// ---------------------------------------------------------------------------------
// Config #3 (BASELINE.json configs[2]): drive-like folder hierarchy.  Folders in `depth`
// levels (level k+1 twice the size of level k), every non-root folder's viewers include
// its parent's: folders:f#viewer@(folders:parent(f)#viewer).  Flat groups with Poisson
// memberships; the remaining tuples are grants folders:f#viewer@(groups:g#member)
// (group_frac) or folders:f#viewer@u.  Checks folders:f#viewer@u, half constructed
// positives (a grant on f or one of its ancestors).  Namespaces: groups 1, folders 2.
typedef struct {
    uint64_t users, groups, folders, tuples, checks, seed;
    double member_mean, group_frac;
    uint64_t depth, check_seed;
} ks_folders_params;

ks_rbac *ks_folders_generate(const ks_folders_params *p) {
    auto *w = new ks_rbac();
    Rng rng(p->seed);
    const uint64_t U = p->users, G = std::max<uint64_t>(p->groups, 1), F = std::max<uint64_t>(p->folders, 1);
    const uint64_t D = std::max<uint64_t>(1, std::min<uint64_t>(p->depth, 30));
    // level sizes: L_k proportional to 2^k
    std::vector<uint64_t> lbase(D + 1, 0);
    {
        double tot = (double)((1ull << D) - 1);
        uint64_t acc = 0;
        for (uint64_t k = 0; k < D; k++) {
            uint64_t sz = k + 1 == D ? F - acc : std::max<uint64_t>(1, (uint64_t)((double)F * (double)(1ull << k) / tot));
            if (acc + sz > F) sz = F - acc;
            lbase[k] = acc;
            acc += sz;
        }
        lbase[D] = F;
    }
    std::vector<uint32_t> parent(F, UINT32_MAX);
    for (uint64_t k = 1; k < D; k++) {
        uint64_t prev = lbase[k] - lbase[k - 1];
        for (uint64_t f = lbase[k]; f < lbase[k + 1]; f++)
            if (prev) parent[f] = (uint32_t)(lbase[k - 1] + rng.below(prev));
    }
    std::vector<std::vector<uint32_t>> members(G);
    std::poisson_distribution<int> pois(p->member_mean);
    std::mt19937_64 mt(p->seed ^ 0x5bd1e995);
    for (uint64_t u = 0; u < U; u++) {
        int k = pois(mt);
        for (int j = 0; j < k; j++) members[rng.below(G)].push_back((uint32_t)u), w->n_member++;
    }
    for (uint64_t f = 0; f < F; f++) w->n_parent += parent[f] != UINT32_MAX;
    uint64_t used = w->n_parent + w->n_member;
    uint64_t n_grant = p->tuples > used ? p->tuples - used : F;
    std::vector<std::vector<uint32_t>> fgroups(F), fusers(F);
    for (uint64_t i = 0; i < n_grant; i++) {
        uint64_t f = rng.below(F);
        if (rng.unit() < p->group_frac)
            fgroups[f].push_back((uint32_t)rng.below(G));
        else
            fusers[f].push_back((uint32_t)rng.below(U));
    }
    w->n_grant = n_grant;
    std::vector<uint32_t> urank(U), grank(G), frank(F);
    {
        auto o = lex_order(U);
        for (uint64_t i = 0; i < U; i++) urank[o[i]] = (uint32_t)i;
        auto og = lex_order(G);
        for (uint64_t i = 0; i < G; i++) grank[og[i]] = (uint32_t)i;
        auto of = lex_order(F);
        for (uint64_t i = 0; i < F; i++) frank[of[i]] = (uint32_t)i;
    }
    auto row_set = [&](int32_t ns, char op, uint64_t o, const char *rel, char sp, uint64_t so, int32_t sns,
                       const char *srel) {
        w->ns.push_back(ns);
        w->kind.push_back(1);
        w->ss_ns.push_back(sns);
        w->obj.put_num(op, o);
        w->rel.put(rel, strlen(rel));
        w->sid.empty();
        w->ss_obj.put_num(sp, so);
        w->ss_rel.put(srel, strlen(srel));
    };
    auto row_id = [&](int32_t ns, char op, uint64_t o, const char *rel, uint64_t u) {
        w->ns.push_back(ns);
        w->kind.push_back(0);
        w->ss_ns.push_back(0);
        w->obj.put_num(op, o);
        w->rel.put(rel, strlen(rel));
        w->sid.put_num('u', u);
        w->ss_obj.empty();
        w->ss_rel.empty();
    };
    auto by_u = [&](uint32_t a, uint32_t b) { return urank[a] < urank[b]; };
    auto by_g = [&](uint32_t a, uint32_t b) { return grank[a] < grank[b]; };
    for (uint32_t g : lex_order(G)) {  // namespace 1: groups
        auto &m = members[g];
        std::sort(m.begin(), m.end(), by_u);
        for (uint32_t u : m) row_id(1, 'g', g, "member", u);
    }
    for (uint32_t f : lex_order(F)) {  // namespace 2: folders; subject sets by (ns id, object)
        auto &fg = fgroups[f];
        std::sort(fg.begin(), fg.end(), by_g);
        for (uint32_t g : fg) row_set(2, 'f', f, "viewer", 'g', g, 1, "member");
        if (parent[f] != UINT32_MAX) row_set(2, 'f', f, "viewer", 'f', parent[f], 2, "viewer");
        auto &fu = fusers[f];
        std::sort(fu.begin(), fu.end(), by_u);
        for (uint32_t u : fu) row_id(2, 'f', f, "viewer", u);
    }
    (void)frank;
    if (p->check_seed) rng = Rng(p->check_seed);
    const uint64_t C = p->checks;
    w->chk_doc.resize(C);
    w->chk_user.resize(C);
    w->chk_pos.resize(C);
    for (uint64_t i = 0; i < C; i++) {
        uint64_t f = rng.below(F), u = rng.below(U);
        bool pos = false;
        if (rng.unit() < 0.5) {
            for (int tries = 0; tries < 64 && !pos; tries++) {
                uint64_t f0 = rng.below(F), a = f0;
                uint64_t up = rng.below(D);
                for (uint64_t s = 0; s < up && parent[a] != UINT32_MAX; s++) a = parent[a];
                uint64_t ng = fgroups[a].size(), nu = fusers[a].size();
                if (!ng && !nu) continue;
                uint64_t k = rng.below(ng + nu);
                if (k >= ng) {
                    f = f0, u = fusers[a][k - ng], pos = true;
                } else {
                    auto &m = members[fgroups[a][k]];
                    if (m.empty()) continue;
                    f = f0, u = m[rng.below(m.size())], pos = true;
                }
            }
        }
        w->chk_doc[i] = (uint32_t)f;
        w->chk_user[i] = (uint32_t)u;
        w->chk_pos[i] = pos;
        w->rq_ns.put("folders", 7);
        w->rq_obj.put_num('f', f);
        w->rq_rel.put("viewer", 6);
        w->rq_sid.put_num('u', u);
    }
    return w;
}

// ---------------------------------------------------------------------------------
// Config #4 (BASELINE.json configs[3]): power-law social/group graph.  Users join
// Poisson(member_mean) groups chosen by Zipf(s) popularity; groups nest into groups
// (groups:gP#member@(groups:gC#member)) with Zipf popularity on BOTH ends, acyclic (the
// parent precedes the child in a random order), `nest_per_group` edges per group on
// average.  Checks groups:g#member@u, g half Zipf-popular half uniform, half constructed
// positives (a walk down from g).  Namespace: groups 1.
typedef struct {
    uint64_t users, groups, tuples, checks, seed;
    double zipf_s, member_mean, nest_per_group;
    uint64_t check_seed;
} ks_social_params;

ks_rbac *ks_social_generate(const ks_social_params *p) {
    auto *w = new ks_rbac();
    Rng rng(p->seed);
    const uint64_t U = p->users, G = std::max<uint64_t>(p->groups, 2);
    std::vector<double> cdf(G);
    {
        double acc = 0;
        for (uint64_t k = 0; k < G; k++) acc += 1.0 / std::pow((double)(k + 1), p->zipf_s), cdf[k] = acc;
        for (auto &x : cdf) x /= acc;
    }
    auto zipf = [&]() {
        uint64_t r = std::lower_bound(cdf.begin(), cdf.end(), rng.unit()) - cdf.begin();
        return r >= G ? G - 1 : r;
    };
    // popularity rank -> group (member side), topological position of each group
    std::vector<uint32_t> pop(G), topo(G), at(G);
    std::iota(pop.begin(), pop.end(), 0u);
    for (uint64_t i = G; i > 1; i--) std::swap(pop[i - 1], pop[rng.below(i)]);
    std::iota(at.begin(), at.end(), 0u);
    for (uint64_t i = G; i > 1; i--) std::swap(at[i - 1], at[rng.below(i)]);
    for (uint64_t i = 0; i < G; i++) topo[at[i]] = (uint32_t)i;  // topo[g] = position
    std::vector<std::vector<uint32_t>> children(G), members(G);
    const uint64_t n_nest = (uint64_t)(p->nest_per_group * (double)G);
    for (uint64_t i = 0; i < n_nest; i++) {
        uint32_t a = pop[zipf()], b = pop[zipf()];
        if (a == b) continue;
        if (topo[a] > topo[b]) std::swap(a, b);  // parent precedes child: acyclic
        children[a].push_back(b);
        w->n_parent++;
    }
    uint64_t budget = p->tuples > w->n_parent ? p->tuples - w->n_parent : U;
    std::poisson_distribution<int> pois(p->member_mean);
    std::mt19937_64 mt(p->seed ^ 0x5bd1e995);
    for (uint64_t u = 0; u < U && w->n_member < budget; u++) {
        int k = pois(mt);
        for (int j = 0; j < k; j++) members[pop[zipf()]].push_back((uint32_t)u), w->n_member++;
    }
    std::vector<uint32_t> urank(U), grank(G);
    {
        auto o = lex_order(U);
        for (uint64_t i = 0; i < U; i++) urank[o[i]] = (uint32_t)i;
        auto og = lex_order(G);
        for (uint64_t i = 0; i < G; i++) grank[og[i]] = (uint32_t)i;
    }
    auto by_u = [&](uint32_t a, uint32_t b) { return urank[a] < urank[b]; };
    auto by_g = [&](uint32_t a, uint32_t b) { return grank[a] < grank[b]; };
    for (uint32_t g : lex_order(G)) {
        auto &ch = children[g];
        std::sort(ch.begin(), ch.end(), by_g);
        for (uint32_t c : ch) {
            w->ns.push_back(1);
            w->kind.push_back(1);
            w->ss_ns.push_back(1);
            w->obj.put_num('g', g);
            w->rel.put("member", 6);
            w->sid.empty();
            w->ss_obj.put_num('g', c);
            w->ss_rel.put("member", 6);
        }
        auto &m = members[g];
        std::sort(m.begin(), m.end(), by_u);
        for (uint32_t u : m) {
            w->ns.push_back(1);
            w->kind.push_back(0);
            w->ss_ns.push_back(0);
            w->obj.put_num('g', g);
            w->rel.put("member", 6);
            w->sid.put_num('u', u);
            w->ss_obj.empty();
            w->ss_rel.empty();
        }
    }
    if (p->check_seed) rng = Rng(p->check_seed);
    const uint64_t C = p->checks;
    w->chk_doc.resize(C);
    w->chk_user.resize(C);
    w->chk_pos.resize(C);
    for (uint64_t i = 0; i < C; i++) {
        uint64_t g = rng.unit() < 0.5 ? pop[zipf()] : rng.below(G), u = rng.below(U);
        bool pos = false;
        if (rng.unit() < 0.5) {
            uint64_t c = g;
            for (int hop = 0; hop < 16 && !pos; hop++) {  // walk down to a member
                uint64_t nc = children[c].size(), nm = members[c].size();
                if (!nc && !nm) break;
                uint64_t k = rng.below(nc + nm);
                if (k >= nc)
                    u = members[c][k - nc], pos = true;
                else
                    c = children[c][k];
            }
        }
        w->chk_doc[i] = (uint32_t)g;
        w->chk_user[i] = (uint32_t)u;
        w->chk_pos[i] = pos;
        w->rq_ns.put("groups", 6);
        w->rq_obj.put_num('g', g);
        w->rq_rel.put("member", 6);
        w->rq_sid.put_num('u', u);
    }
    return w;
}

// ---------------------------------------------------------------------------------
// Config #5 (BASELINE.json configs[4]): the config #2 RBAC shape at 5B tuples, for the
// hash-partitioned mode.  Too large to materialize (the rows alone are ~150 GB), so the
// graph is defined node by node by counter-based random draws — the k-th child of group
// j, the k-th member of leaf group j, the k-th grant of doc d are pure functions of
// (seed, node, k) — and STREAMED in the reference's ORDER BY order (SQLite semantics),
// batch by batch, without holding more than one group's rows.  Every rank of the
// partitioned loader runs the same stream.  Shape: groups in 4 levels (1/4/15/80 %);
// a group of level l < 3 has floor(lambda + u) children drawn from level l + 1
// (lambda = 1.5 |L_{l+1}| / |L_l|); leaf group j has floor(M w(j) + u) members, w = Zipf(s)
// over a fixed permutation of the leaves, M = users * member_mean; doc d has
// floor(lambda_g + u) grants, 80 % to a group, 20 % to a user, lambda_g filling the
// tuple budget.  Checks docs:d#viewer@u: half constructed positives (a grant path walked
// down by random access), half uniform pairs.
typedef struct {
    uint64_t users, groups, docs, tuples, seed;
    double zipf_s, member_mean;
} ks_c5_params;

namespace {

inline uint64_t cmix(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// decimal-string order of numbers < 10^10: n * 10^(10 - digits) with the digit count as
// tie-break (a prefix sorts first)
inline uint64_t lex_key(uint64_t n) {
    int d = 1;
    uint64_t p = 10;
    while (n >= p && d < 10) d++, p *= 10;
    uint64_t k = n;
    for (int i = d; i < 10; i++) k *= 10;
    return k * 16 + (uint64_t)d;
}

// numbers 0..n-1 in the order of their decimal strings, without a table
struct LexIter {
    uint64_t n = 0, cur = 0;
    bool started = false, done = false;
    void reset(uint64_t n_) {
        n = n_;
        cur = 0;
        started = false;
        done = n == 0;
    }
    bool next(uint64_t &out) {
        if (done) return false;
        if (!started) {
            started = true;
            cur = 0;
            out = 0;
            if (n <= 1) done = true;
            return true;
        }
        if (cur == 0) {
            cur = 1;
        } else if (cur * 10 < n) {
            cur *= 10;
        } else {
            while (cur % 10 == 9 || cur + 1 >= n) {
                cur /= 10;
                if (cur == 0) {
                    done = true;
                    return false;
                }
            }
            cur += 1;
        }
        out = cur;
        return true;
    }
};

}  // namespace

struct ks_c5 {
    ks_c5_params p{};
    uint64_t base[5] = {0, 0, 0, 0, 0}, lv[4] = {0, 0, 0, 0};
    double lam_child[3] = {0, 0, 0}, lam_grant = 0, zipf_h = 0, members = 0;
    uint64_t perm_a = 1, perm_b = 0;
    // stream state
    int phase = 0;  // 0 groups, 1 docs, 2 done
    LexIter it;
    std::vector<uint64_t> cur_sets, cur_users;  // lex keys of the current node's subjects
    uint64_t cur_obj = 0, cur_pos = 0;
    bool cur_open = false;
    ks_rbac batch;  // the last batch's columns (and the checks)
    uint64_t rows_out = 0;

    uint64_t draw(uint64_t node_tag, uint64_t stream, uint64_t k) const {
        return cmix(p.seed ^ cmix(node_tag * 0x9e3779b97f4a7c15ull + stream) ^ (k * 0xd1b54a32d192ed03ull));
    }
    double unit(uint64_t x) const { return (x >> 11) * (1.0 / 9007199254740992.0); }
    int level(uint64_t g) const { return g < base[1] ? 0 : g < base[2] ? 1 : g < base[3] ? 2 : 3; }
    uint64_t count(uint64_t tag, double lam) const { return (uint64_t)(lam + unit(draw(tag, 0, 0))); }
    // group j: children (groups of the next level) and members (users, leaves only)
    uint64_t n_children(uint64_t g) const {
        const int l = level(g);
        return l < 3 ? count(g * 4 + 1, lam_child[l]) : 0;
    }
    uint64_t child(uint64_t g, uint64_t k) const {
        const int l = level(g);
        return base[l + 1] + draw(g * 4 + 1, 1, k) % lv[l + 1];
    }
    uint64_t n_members(uint64_t g) const {
        if (level(g) != 3) return 0;
        const uint64_t rank = (perm_a * (g - base[3]) + perm_b) % lv[3];
        const double w = 1.0 / std::pow((double)(rank + 1), p.zipf_s) / zipf_h;
        return count(g * 4 + 2, members * w);
    }
    uint64_t member(uint64_t g, uint64_t k) const { return draw(g * 4 + 2, 2, k) % p.users; }
    // doc d: grants, 80 % to a group
    uint64_t n_grants(uint64_t d) const { return count(d * 4 + 3, lam_grant); }
    bool grant_group(uint64_t d, uint64_t k) const { return unit(draw(d * 4 + 3, 3, k)) < 0.8; }
    uint64_t grant_target(uint64_t d, uint64_t k) const {
        return draw(d * 4 + 3, 4, k) % (grant_group(d, k) ? p.groups : p.users);
    }

    void init(const ks_c5_params &q) {
        p = q;
        const uint64_t G = std::max<uint64_t>(p.groups, 4), U = std::max<uint64_t>(p.users, 1);
        p.groups = G;
        p.users = U;
        p.docs = std::max<uint64_t>(p.docs, 1);
        lv[0] = std::max<uint64_t>(1, G / 100);
        lv[1] = std::max<uint64_t>(1, G * 4 / 100);
        lv[2] = std::max<uint64_t>(1, G * 15 / 100);
        lv[3] = G - lv[0] - lv[1] - lv[2];
        for (int l = 0; l < 4; l++) base[l + 1] = base[l] + lv[l];
        for (int l = 0; l < 3; l++) lam_child[l] = 1.5 * (double)lv[l + 1] / (double)lv[l];
        for (uint64_t k = 0; k < lv[3]; k++) zipf_h += 1.0 / std::pow((double)(k + 1), p.zipf_s);
        members = (double)U * p.member_mean;
        perm_a = (cmix(p.seed) | 1) % lv[3];
        while (std::gcd(perm_a, lv[3]) != 1) perm_a++;
        perm_b = cmix(p.seed + 1) % lv[3];
        double used = members;
        for (int l = 0; l < 3; l++) used += lam_child[l] * (double)lv[l];
        lam_grant = std::max(0.0, ((double)p.tuples - used) / (double)p.docs);
        rewind();
    }
    void rewind() {
        phase = 0;
        it.reset(p.groups);
        cur_open = false;
        rows_out = 0;
    }
    // the next node's rows, sorted as the ORDER BY sorts them (subject sets first)
    bool open_next() {
        uint64_t o;
        while (phase < 2) {
            if (it.next(o)) {
                cur_obj = o;
                cur_sets.clear();
                cur_users.clear();
                if (phase == 0) {
                    for (uint64_t k = 0, n = n_children(o); k < n; k++) cur_sets.push_back(lex_key(child(o, k)));
                    for (uint64_t k = 0, n = n_members(o); k < n; k++) cur_users.push_back(lex_key(member(o, k)));
                } else {
                    for (uint64_t k = 0, n = n_grants(o); k < n; k++)
                        (grant_group(o, k) ? cur_sets : cur_users).push_back(lex_key(grant_target(o, k)));
                }
                if (cur_sets.empty() && cur_users.empty()) continue;
                std::sort(cur_sets.begin(), cur_sets.end());
                std::sort(cur_users.begin(), cur_users.end());
                cur_pos = 0;
                cur_open = true;
                return true;
            }
            phase++;
            if (phase == 1) it.reset(p.docs);
        }
        return false;
    }
    static uint64_t unkey(uint64_t k) {
        const int d = (int)(k & 15);
        k >>= 4;
        for (int i = d; i < 10; i++) k /= 10;
        return k;
    }
    uint64_t next_batch(uint64_t max_rows) {
        ks_rbac &w = batch;
        w.ns.clear();
        w.ss_ns.clear();
        w.kind.clear();
        for (Col *c : {&w.obj, &w.rel, &w.sid, &w.ss_obj, &w.ss_rel}) {
            c->data.clear();
            c->off.assign(1, 0);
        }
        uint64_t n = 0;
        while (n < max_rows) {
            if (!cur_open && !open_next()) break;
            const bool doc = phase == 1;
            const uint64_t ns_sets = cur_sets.size(), total = ns_sets + cur_users.size();
            for (; cur_pos < total && n < max_rows; cur_pos++, n++) {
                w.ns.push_back(doc ? 2 : 1);
                w.obj.put_num(doc ? 'd' : 'g', cur_obj);
                if (doc)
                    w.rel.put("viewer", 6);
                else
                    w.rel.put("member", 6);
                if (cur_pos < ns_sets) {
                    w.kind.push_back(1);
                    w.ss_ns.push_back(1);
                    w.sid.empty();
                    w.ss_obj.put_num('g', unkey(cur_sets[cur_pos]));
                    w.ss_rel.put("member", 6);
                } else {
                    w.kind.push_back(0);
                    w.ss_ns.push_back(0);
                    w.sid.put_num('u', unkey(cur_users[cur_pos - ns_sets]));
                    w.ss_obj.empty();
                    w.ss_rel.empty();
                }
            }
            if (cur_pos == total) cur_open = false;
        }
        rows_out += n;
        return n;
    }
    void checks(uint64_t C, uint64_t check_seed) {
        ks_rbac &w = batch;
        Rng rng(check_seed ? check_seed : p.seed + 1);
        w.chk_doc.resize(C);
        w.chk_user.resize(C);
        w.chk_pos.resize(C);
        w.rq_ns = w.rq_obj = w.rq_rel = w.rq_sid = Col();
        for (uint64_t i = 0; i < C; i++) {
            uint64_t d = rng.below(p.docs), u = rng.below(p.users);
            bool pos = false;
            if (rng.unit() < 0.5) {
                for (int tries = 0; tries < 64 && !pos; tries++) {  // a grant path, walked down
                    const uint64_t dd = rng.below(p.docs), ng = n_grants(dd);
                    if (!ng) continue;
                    const uint64_t k = rng.below(ng);
                    if (!grant_group(dd, k)) {
                        d = dd, u = grant_target(dd, k), pos = true;
                        break;
                    }
                    uint64_t g = grant_target(dd, k);
                    for (int hop = 0; hop < 8; hop++) {
                        const uint64_t nc = n_children(g), nm = n_members(g);
                        if (!nc && !nm) break;
                        const uint64_t j = rng.below(nc + nm);
                        if (j >= nc) {
                            d = dd, u = member(g, j - nc), pos = true;
                            break;
                        }
                        g = child(g, j);
                    }
                }
            }
            w.chk_doc[i] = (uint32_t)d;
            w.chk_user[i] = (uint32_t)u;
            w.chk_pos[i] = pos;
            w.rq_ns.put("docs", 4);
            w.rq_obj.put_num('d', d);
            w.rq_rel.put("viewer", 6);
            w.rq_sid.put_num('u', u);
        }
    }
};

ks_c5 *ks_c5_new(const ks_c5_params *p) {
    auto *g = new ks_c5();
    g->init(*p);
    return g;
}
void ks_c5_rewind(ks_c5 *g) { g->rewind(); }
// the next batch of at most max_rows rows into the generator's column buffers (valid until
// the next call); 0 at the end of the stream
uint64_t ks_c5_next(ks_c5 *g, uint64_t max_rows) { return g->next_batch(max_rows); }
void ks_c5_checks(ks_c5 *g, uint64_t checks, uint64_t check_seed) { g->checks(checks, check_seed); }
ks_rbac *ks_c5_buffers(ks_c5 *g) { return &g->batch; }
void ks_c5_free(ks_c5 *g) { delete g; }

void ks_rbac_view_get(const ks_rbac *w, ks_rbac_view *v) {
    v->n = w->ns.size();
    v->namespace_id = w->ns.data();
    v->object_data = w->obj.data.data();
    v->object_off = w->obj.off.data();
    v->relation_data = w->rel.data.data();
    v->relation_off = w->rel.off.data();
    v->subject_kind = w->kind.data();
    v->subject_id_data = w->sid.data.data();
    v->subject_id_off = w->sid.off.data();
    v->ss_namespace_id = w->ss_ns.data();
    v->ss_object_data = w->ss_obj.data.data();
    v->ss_object_off = w->ss_obj.off.data();
    v->ss_relation_data = w->ss_rel.data.data();
    v->ss_relation_off = w->ss_rel.off.data();
    v->n_checks = w->chk_doc.size();
    v->chk_doc = w->chk_doc.data();
    v->chk_user = w->chk_user.data();
    v->chk_pos = w->chk_pos.data();
    v->rq_ns_data = w->rq_ns.data.data();
    v->rq_ns_off = w->rq_ns.off.data();
    v->rq_obj_data = w->rq_obj.data.data();
    v->rq_obj_off = w->rq_obj.off.data();
    v->rq_rel_data = w->rq_rel.data.data();
    v->rq_rel_off = w->rq_rel.off.data();
    v->rq_sid_data = w->rq_sid.data.data();
    v->rq_sid_off = w->rq_sid.off.data();
    v->n_parent = w->n_parent;
    v->n_member = w->n_member;
    v->n_grant = w->n_grant;
}

void ks_rbac_free(ks_rbac *w) { delete w; }

}  // extern "C"
