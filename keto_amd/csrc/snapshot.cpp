// snapshot.cpp — persistence-side snapshot loader (new component; replaces the
// per-node SQL reads of (*Persister).GetRelationTuples,
// internal/persistence/sql/relationtuples.go:203-258).
//
// Input: keto_relation_tuples rows of one network in the backend's ORDER BY order
// (relationtuples.go:215), streamed in columnar batches.  Output: a Snapshot with
//   * per-group row lists in DB order (expand needs the order, R9),
//   * interned subject nodes and, per subject set, its query's rows after applying the
//     reference's empty-field wildcards (R5) and page-poison truncation (R7),
//   * the device graph: forward interior CSR + reverse CSR (check needs reachability
//     only), and the ambiguous-key bitmap (R4).
#include <algorithm>
#include <chrono>
#include <numeric>

#include "ketogpu_internal.hpp"

namespace ketogpu {

// ------------------------------------------------------------------ StrPool
uint32_t StrPool::find(const char *p, size_t n) const {
    if (!mask_) return NONE;
    uint64_t h = hash_bytes(p, n);
    for (size_t j = h & mask_;; j = (j + 1) & mask_) {
        uint32_t id = slot_id_[j];
        if (!id) return NONE;
        if (slot_hash_[j] == h && len_[id - 1] == n && !memcmp(ptr_[id - 1], p, n)) return id - 1;
    }
}

void StrPool::rehash() {
    size_t cap = slot_id_.empty() ? 1024 : slot_id_.size() * 2;
    std::vector<uint64_t> nh(cap);
    std::vector<uint32_t> ni(cap, 0);
    size_t m = cap - 1;
    for (size_t j = 0; j < slot_id_.size(); j++)
        if (slot_id_[j]) {
            size_t k = slot_hash_[j] & m;
            while (ni[k]) k = (k + 1) & m;
            nh[k] = slot_hash_[j];
            ni[k] = slot_id_[j];
        }
    slot_hash_.swap(nh);
    slot_id_.swap(ni);
    mask_ = m;
}

uint32_t StrPool::intern(const char *p, size_t n) {
    if ((ptr_.size() + 1) * 2 > slot_id_.size()) rehash();
    uint64_t h = hash_bytes(p, n);
    size_t j = h & mask_;
    for (;; j = (j + 1) & mask_) {
        uint32_t id = slot_id_[j];
        if (!id) break;
        if (slot_hash_[j] == h && len_[id - 1] == n && !memcmp(ptr_[id - 1], p, n)) return id - 1;
    }
    if (used_ + n + 1 > cap_) {
        cap_ = std::max<size_t>(n + 1, (size_t)1 << 22);
        chunks_.emplace_back(new char[cap_]);
        used_ = 0;
    }
    char *dst = chunks_.back().get() + used_;
    memcpy(dst, p, n);
    dst[n] = 0;
    used_ += n + 1;
    uint32_t id = (uint32_t)ptr_.size();
    ptr_.push_back(dst);
    len_.push_back((uint32_t)n);
    slot_hash_[j] = h;
    slot_id_[j] = id + 1;
    return id;
}

// ---------------------------------------------------------------- TripleMap
void TripleMap::resize(size_t cap) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(cap, Slot{0, 0, 0, NONE});
    mask_ = cap - 1;
    n_ = 0;
    for (auto &s : old)
        if (s.val != NONE) get_or_insert(s.ns, s.obj, s.rel, s.val);
}

uint32_t TripleMap::get(int32_t ns, uint32_t obj, uint32_t rel) const {
    for (size_t j = h(ns, obj, rel) & mask_;; j = (j + 1) & mask_) {
        const Slot &s = slots_[j];
        if (s.val == NONE) return NONE;
        if (s.ns == ns && s.obj == obj && s.rel == rel) return s.val;
    }
}

uint32_t TripleMap::get_or_insert(int32_t ns, uint32_t obj, uint32_t rel, uint32_t v) {
    if ((n_ + 1) * 2 > slots_.size()) resize(slots_.size() * 2);
    for (size_t j = h(ns, obj, rel) & mask_;; j = (j + 1) & mask_) {
        Slot &s = slots_[j];
        if (s.val == NONE) {
            s = Slot{ns, obj, rel, v};
            n_++;
            return v;
        }
        if (s.ns == ns && s.obj == obj && s.rel == rel) return s.val;
    }
}

void TripleMap::remap(const std::vector<uint32_t> &perm) {
    for (auto &s : slots_)
        if (s.val != NONE) s.val = perm[s.val];
}

// ----------------------------------------------------------------- Snapshot
std::string Snapshot::key_string(uint32_t v) const {
    // Subject.String() (internal/relationtuple/definitions.go:164-170)
    if (node_kind[v] == KETOGPU_SUBJECT_ID) return std::string(pool.get(node_a[v]));
    const Namespace *n = ns_by_id(node_ns[v]);
    std::string k(n ? n->name : std::string());
    k += ':';
    k += pool.get(node_a[v]);
    k += '#';
    k += pool.get(node_b[v]);
    return k;
}

RowRef Snapshot::materialize(bool any_ns, int32_t ns, uint32_t obj, bool any_obj, uint32_t rel,
                             bool any_rel, std::vector<uint32_t> &out) const {
    // The rows a GetRelationTuples query returns, page after page, are the matching
    // groups' rows in group order, because ORDER BY starts with
    // (namespace_id, object, relation).  The first page holding a row whose namespace
    // id is unknown fails (toInternal), so the check engine sees only the complete pages
    // before it (engine.go:74-77): truncate at page_size * floor(first_bad / page_size).
    RowRef r;
    r.off = out.size();
    uint64_t total = 0;
    int64_t bad = -1;
    for (const Group &g : groups) {
        if (!any_ns && g.ns != ns) continue;
        if (!any_obj && g.obj != obj) continue;
        if (!any_rel && g.rel != rel) continue;
        if (bad < 0) {
            out.insert(out.end(), group_col.begin() + g.begin, group_col.begin() + g.begin + g.valid);
            if (g.first_bad >= 0) bad = (int64_t)total + g.first_bad;
        }
        total += g.full_len;
    }
    uint64_t keep = out.size() - r.off;
    if (bad >= 0) {
        uint64_t t = (uint64_t)(bad / page_size) * (uint64_t)page_size;
        if (t < keep) keep = t;
        out.resize(r.off + keep);
    }
    r.len = (uint32_t)keep;
    r.full_len = (uint32_t)std::min<uint64_t>(total, 0xffffffffu);
    r.first_bad = bad;
    return r;
}

}  // namespace ketogpu

using namespace ketogpu;

// ------------------------------------------------------------------ builder
struct ketogpu_builder {
    std::unique_ptr<Snapshot> s;
    uint32_t flags = 0;
    std::chrono::steady_clock::time_point t0;
    // streaming group state
    bool open = false;
    Group cur{};
    std::string cur_obj, cur_rel;  // raw bytes of the open group (fast path)
    TripleMap seen_groups;         // detects rows that are not grouped
    // KETOGPU_BUILD_SORT: rows buffered as interned ids
    using RawRow = TupleRow;
    std::vector<RawRow> raw;
    uint64_t rows = 0, bad_rows = 0;
    std::vector<uint8_t> ns_known_dense;  // namespace ids in [0, 65536) fast path

    bool ns_known(int32_t id) const {
        if (id >= 0 && id < (int32_t)ns_known_dense.size()) return ns_known_dense[id];
        return s->ns_by_id(id) != nullptr;
    }
    uint32_t id_node(uint32_t sid_str) {
        Snapshot &S = *s;
        if (S.sid_node.size() <= sid_str) S.sid_node.resize(std::max<size_t>(sid_str + 1, S.sid_node.size() * 2), NONE);
        uint32_t &v = S.sid_node[sid_str];
        if (v == NONE) {
            v = (uint32_t)S.node_kind.size();
            S.node_kind.push_back(KETOGPU_SUBJECT_ID);
            S.node_ns.push_back(0);
            S.node_a.push_back(sid_str);
            S.node_b.push_back(0);
        }
        return v;
    }
    uint32_t set_node(int32_t ns, uint32_t obj, uint32_t rel) {
        Snapshot &S = *s;
        uint32_t nv = (uint32_t)S.node_kind.size();
        uint32_t v = S.set_node.get_or_insert(ns, obj, rel, nv);
        if (v == nv) {
            S.node_kind.push_back(KETOGPU_SUBJECT_SET);
            S.node_ns.push_back(ns);
            S.node_a.push_back(obj);
            S.node_b.push_back(rel);
        }
        return v;
    }
    void close_group() {
        if (!open) return;
        s->groups.push_back(cur);
        open = false;
    }
    void open_group(int32_t ns, uint32_t obj, uint32_t rel) {
        if (seen_groups.get(ns, obj, rel) != NONE)
            throw Error(KETOGPU_EINVAL,
                        "rows are not in ORDER BY order: group (namespace_id, object, relation) "
                        "appears twice (use KETOGPU_BUILD_SORT)");
        seen_groups.get_or_insert(ns, obj, rel, (uint32_t)s->groups.size());
        cur = Group{ns, obj, rel, 0, s->group_col.size(), 0, 0, -1, 0};
        open = true;
    }
    // one row, already grouped
    void add(int32_t ns, uint32_t obj, uint32_t rel, uint8_t kind, uint32_t sid, int32_t ss_ns,
             uint32_t ss_obj, uint32_t ss_rel) {
        if (!open || cur.ns != ns || cur.obj != obj || cur.rel != rel) {
            close_group();
            open_group(ns, obj, rel);
        }
        rows++;
        // toInternal fails for unknown namespace ids (relationtuples.go:48-51,64-67)
        bool bad = !ns_known(ns) || (kind && !ns_known(ss_ns));
        if (bad) bad_rows++;
        if (cur.first_bad < 0 && bad) {
            cur.first_bad = cur.full_len;
            cur.tail = s->tail_rows.size();
        }
        if (cur.first_bad < 0) {
            uint32_t v = kind ? set_node(ss_ns, ss_obj, ss_rel) : id_node(sid);
            s->group_col.push_back(v);
            cur.valid++;
        } else {  // invisible to check/expand past the poisoned page, kept for updates
            s->tail_rows.push_back(TupleRow{ns, ss_ns, obj, rel, sid, ss_obj, ss_rel, kind, 0});
        }
        cur.full_len++;
    }
};

namespace {

inline std::string_view col(const char *data, const uint64_t *off, size_t i) {
    if (!data || !off) return std::string_view();
    return std::string_view(data + off[i], off[i + 1] - off[i]);
}

// The backend's ORDER BY (relationtuples.go:215) for KETOGPU_BUILD_SORT and apply: bytewise
// strings; NULLs first (SQLite, MySQL binary collations, CockroachDB) or last (Postgres,
// KETOGPU_ORDER_NULLS_LAST).  Only subject_id is NULL for some rows of a group (subject-set
// rows), so NULL placement decides whether subject sets or subject ids come first.
struct SortCmp {
    const StrPool &p;
    bool nulls_last = false;
    int cs(uint32_t a, uint32_t b) const {
        if (a == b) return 0;
        std::string_view x = p.get(a), y = p.get(b);
        int c = memcmp(x.data(), y.data(), std::min(x.size(), y.size()));
        if (c) return c;
        return x.size() < y.size() ? -1 : (x.size() > y.size());
    }
    bool operator()(const ketogpu_builder::RawRow &a, const ketogpu_builder::RawRow &b) const {
        if (a.ns != b.ns) return a.ns < b.ns;
        int c;
        if ((c = cs(a.obj, b.obj))) return c < 0;
        if ((c = cs(a.rel, b.rel))) return c < 0;
        if (a.kind != b.kind) return nulls_last ? a.kind < b.kind : a.kind > b.kind;  // NULL subject_id = set row
        if (!a.kind) {
            if ((c = cs(a.sid, b.sid))) return c < 0;
        } else {
            if (a.ss_ns != b.ss_ns) return a.ss_ns < b.ss_ns;
            if ((c = cs(a.ss_obj, b.ss_obj))) return c < 0;
            if ((c = cs(a.ss_rel, b.ss_rel))) return c < 0;
        }
        return a.seq < b.seq;
    }
};

void finish_snapshot(ketogpu_builder *b) {
    Snapshot &S = *b->s;
    if (b->flags & KETOGPU_BUILD_SORT) {
        std::stable_sort(b->raw.begin(), b->raw.end(), SortCmp{S.pool, S.nulls_last});
        for (auto &r : b->raw) b->add(r.ns, r.obj, r.rel, r.kind, r.sid, r.ss_ns, r.ss_obj, r.ss_rel);
        std::vector<ketogpu_builder::RawRow>().swap(b->raw);
    }
    b->close_group();

    // every group of a configured namespace is a subject-set node (it can be a root and
    // a target even if nothing points at it)
    for (const Group &g : S.groups)
        if (b->ns_known(g.ns)) b->set_node(g.ns, g.obj, g.rel);

    // writable layout: three placeholder nodes (no name, no rows) that pad device rows
    // (ketogpu_internal.hpp, snapshot_write.cpp); created last so they take the largest ids
    // of their classes
    const bool writable = (b->flags & KETOGPU_BUILD_WRITABLE) != 0;
    uint32_t ph[3] = {NONE, NONE, NONE};  // Dbi, Df (interior), Dbo (expandable)
    if (writable)
        for (uint32_t &x : ph) {
            x = (uint32_t)S.node_kind.size();
            S.node_kind.push_back(KETOGPU_SUBJECT_ID);
            S.node_ns.push_back(0);
            S.node_a.push_back(0);
            S.node_b.push_back(0);
        }
    const uint32_t N = (uint32_t)S.node_kind.size();
    const size_t ps = (size_t)S.page_size;
    std::vector<RowRef> row(N);
    std::vector<uint32_t> group_of(N, NONE);
    for (uint32_t gi = 0; gi < S.groups.size(); gi++) {
        const Group &g = S.groups[gi];
        if (!b->ns_known(g.ns)) continue;
        group_of[S.set_node.get(g.ns, g.obj, g.rel)] = gi;
    }
    // rows of every subject-set node: concrete queries reference their group, queries
    // with an empty field (or the namespace named "") are materialized (R5)
    std::vector<uint32_t> &rc = S.row_col;
    rc = S.group_col;  // row_col starts with the groups' valid prefixes
    uint64_t wild = 0;
    for (uint32_t v = 0; v < N; v++) {
        if (S.node_kind[v] != KETOGPU_SUBJECT_SET) continue;
        const Namespace *n = S.ns_by_id(S.node_ns[v]);
        bool any_ns = n && n->name.empty();
        bool any_obj = S.node_a[v] == 0, any_rel = S.node_b[v] == 0;  // pool id 0 == ""
        if (any_ns || any_obj || any_rel) {
            wild++;
            row[v] = S.materialize(any_ns, S.node_ns[v], S.node_a[v], any_obj, S.node_b[v], any_rel, rc);
        } else if (group_of[v] != NONE) {
            const Group &g = S.groups[group_of[v]];
            RowRef r;
            r.off = g.begin;
            r.full_len = g.full_len;
            r.first_bad = g.first_bad;
            r.len = g.valid;
            if (g.first_bad >= 0) r.len = (uint32_t)std::min<uint64_t>(g.valid, (g.first_bad / ps) * ps);
            row[v] = r;
        }
    }

    // classify: expandable = non-empty rows; interior = expandable and a subject of
    // some expandable node's rows
    std::vector<uint8_t> cls(N, 2);  // 0 interior, 1 source, 2 non-expandable
    for (uint32_t v = 0; v < N; v++)
        if (row[v].len) cls[v] = 1;
    for (uint32_t v = 0; v < N; v++) {
        if (!row[v].len) continue;
        const uint32_t *p = rc.data() + row[v].off;
        for (uint32_t i = 0; i < row[v].len; i++)
            if (cls[p[i]] == 1) cls[p[i]] = 0;
    }
    if (writable) cls[ph[0]] = cls[ph[1]] = 0, cls[ph[2]] = 1;
    std::vector<uint32_t> perm(N), inv(N);
    {
        uint32_t c[3] = {0, 0, 0};
        for (uint32_t v = 0; v < N; v++) c[cls[v]]++;
        S.Ni = c[0];
        S.Nx = c[0] + c[1];
        S.N = N;
        uint32_t base[3] = {0, c[0], c[0] + c[1]};
        for (uint32_t v = 0; v < N; v++) perm[v] = base[cls[v]]++;
        for (uint32_t v = 0; v < N; v++) inv[perm[v]] = v;
    }
    // apply the permutation
    for (auto &x : rc) x = perm[x];
    for (auto &x : S.group_col) x = perm[x];
    for (auto &x : S.sid_node)
        if (x != NONE) x = perm[x];
    S.set_node.remap(perm);
    if (writable) S.writable = true, S.Dbi = perm[ph[0]], S.Df = perm[ph[1]], S.Dbo = perm[ph[2]];
    {
        std::vector<uint8_t> k(N);
        std::vector<int32_t> ns(N);
        std::vector<uint32_t> a(N), bb(N);
        std::vector<RowRef> r(N);
        for (uint32_t nv = 0; nv < N; nv++) {
            uint32_t o = inv[nv];
            k[nv] = S.node_kind[o];
            ns[nv] = S.node_ns[o];
            a[nv] = S.node_a[o];
            bb[nv] = S.node_b[o];
            r[nv] = row[o];
        }
        S.node_kind.swap(k);
        S.node_ns.swap(ns);
        S.node_a.swap(a);
        S.node_b.swap(bb);
        S.node_row.swap(r);
    }

    // Subject.String() identities (R4).  Two distinct nodes can share a key only if a
    // subject-set field contains ':' or '#', or a subject id contains both; keys of all
    // other subject ids are unique without building the string.
    S.key_id.assign(N, 0);
    S.ambiguous.assign(N, 0);
    {
        StrPool &keys = S.key_pool;
        std::vector<uint32_t> first(1, NONE);
        uint64_t amb = 0;
        for (uint32_t v = 0; v < N; v++) {
            bool need = S.node_kind[v] == KETOGPU_SUBJECT_SET;
            if (!need) {
                std::string_view id = S.pool.get(S.node_a[v]);
                need = id.find(':') != std::string_view::npos && id.find('#') != std::string_view::npos;
            }
            if (!need) {
                S.key_id[v] = 0x80000000u | v;
                continue;
            }
            std::string k = S.key_string(v);
            uint32_t kid = keys.intern(k.data(), k.size());
            if (first.size() <= kid) first.resize(kid + 1, NONE);
            if (first[kid] == NONE) {
                first[kid] = v;
            } else {
                if (!S.ambiguous[first[kid]]) amb++, S.ambiguous[first[kid]] = 1;
                if (!S.ambiguous[v]) amb++, S.ambiguous[v] = 1;
            }
            S.key_id[v] = kid;
        }
        S.has_ambiguous = amb > 0;
        S.stats.num_ambiguous_nodes = amb;
    }

    // device graph: forward interior CSR over [0, Nx) and reverse CSR over [0, N)
    const uint32_t Ni = S.Ni, Nx = S.Nx;
    S.fint_off.assign((size_t)Nx + 1, 0);
    S.rev_off.assign((size_t)N + 1, 0);
    S.row_amb.assign(((size_t)Nx + 31) / 32, 0);
    std::vector<uint32_t> mark(N, NONE);
    uint64_t nint = 0, nrev = 0;
    for (uint32_t v = 0; v < Nx; v++) {
        const uint32_t *p = S.row_ptr(v);
        for (uint32_t i = 0; i < S.node_row[v].len; i++) {
            uint32_t u = p[i];
            if (S.ambiguous[u]) S.row_amb[v >> 5] |= 1u << (v & 31);
            if (mark[u] == v) continue;
            mark[u] = v;
            S.rev_off[u + 1]++;
            nrev++;
            if (u < Ni) S.fint_off[v + 1]++, nint++;
        }
    }
    for (uint32_t v = 0; v < Nx; v++) S.fint_off[v + 1] += S.fint_off[v];
    for (uint32_t u = 0; u < N; u++) S.rev_off[u + 1] += S.rev_off[u];
    S.fint_col.resize(nint);
    S.rev_col.resize(nrev);
    {
        std::vector<uint64_t> rpos(S.rev_off.begin(), S.rev_off.end() - 1);
        std::fill(mark.begin(), mark.end(), NONE);
        for (uint32_t v = 0; v < Nx; v++) {
            const uint32_t *p = S.row_ptr(v);
            uint64_t fp = S.fint_off[v];
            for (uint32_t i = 0; i < S.node_row[v].len; i++) {
                uint32_t u = p[i];
                if (mark[u] == v) continue;
                mark[u] = v;
                S.rev_col[rpos[u]++] = v;  // ascending v: reverse lists come out sorted
                if (u < Ni) S.fint_col[fp++] = u;
            }
            std::sort(S.fint_col.begin() + S.fint_off[v], S.fint_col.begin() + S.fint_off[v + 1]);
        }
    }

    auto &st = S.stats;
    st.num_rows = b->rows;
    st.num_bad_rows = b->bad_rows;
    st.num_groups = S.groups.size();
    st.num_nodes = N;
    st.num_expandable = Nx;
    st.num_interior = Ni;
    uint64_t edges = 0;
    for (uint32_t v = 0; v < Nx; v++) edges += S.node_row[v].len;
    st.num_edges = edges;
    st.num_interior_edges = nint;
    st.num_rev_edges = nrev;
    st.num_wildcard_nodes = wild;
    if (writable) make_writable(S);
    st.build_seconds =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - b->t0).count();
}

}  // namespace

// ------------------------------------------------------------------- C ABI
extern "C" {

int ketogpu_builder_new(const ketogpu_namespace *namespaces, size_t num_namespaces,
                        const ketogpu_build_opts *opts, ketogpu_builder **out) {
    try {
        *out = nullptr;
        auto b = std::make_unique<ketogpu_builder>();
        b->t0 = std::chrono::steady_clock::now();
        b->s = std::make_unique<Snapshot>();
        Snapshot &S = *b->s;
        for (size_t i = 0; i < num_namespaces; i++) {
            Namespace n{namespaces[i].id, namespaces[i].name ? namespaces[i].name : ""};
            // the reference resolves names and ids by first match (namespace_memory.go:29-47);
            // duplicates would make a subject set's identity depend on that scan order
            for (auto &m : S.namespaces)
                if (m.id == n.id || m.name == n.name)
                    throw Error(KETOGPU_EINVAL, "duplicate namespace name or id in configuration: " + n.name);
            S.namespaces.push_back(n);
            if (n.name.empty()) S.has_empty_name_ns = true, S.empty_name_ns = n.id;
            if (n.id >= 0 && n.id < 65536) {
                if ((int32_t)b->ns_known_dense.size() <= n.id) b->ns_known_dense.resize(n.id + 1, 0);
                b->ns_known_dense[n.id] = 1;
            }
        }
        if (opts) {
            if (opts->page_size < 0) throw Error(KETOGPU_EINVAL, "negative page size");
            if (opts->page_size) S.page_size = opts->page_size;
            if (opts->flags & ~(KETOGPU_BUILD_SORT | KETOGPU_ORDER_NULLS_LAST | KETOGPU_BUILD_WRITABLE))
                throw Error(KETOGPU_EINVAL, "unknown builder flags");
            b->flags = opts->flags;
            S.nulls_last = (opts->flags & KETOGPU_ORDER_NULLS_LAST) != 0;
        }
        *out = b.release();
        return KETOGPU_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
}

int ketogpu_builder_append(ketogpu_builder *b, const ketogpu_row_batch *r) {
    try {
        if (!b || !r) throw Error(KETOGPU_EINVAL, "null argument");
        if (!r->n) return KETOGPU_OK;
        if (!r->namespace_id || !r->object_off || !r->relation_off || !r->subject_kind)
            throw Error(KETOGPU_EINVAL, "row batch misses a required column");
        Snapshot &S = *b->s;
        uint32_t last_obj = 0, last_rel = 0;
        for (size_t i = 0; i < r->n; i++) {
            std::string_view obj = col(r->object_data, r->object_off, i);
            std::string_view rel = col(r->relation_data, r->relation_off, i);
            // fast path: consecutive rows of one group repeat object and relation
            uint32_t oid, rid;
            if (b->open && obj == b->cur_obj && rel == b->cur_rel && !(b->flags & KETOGPU_BUILD_SORT)) {
                oid = b->cur.obj;
                rid = b->cur.rel;
            } else {
                oid = S.pool.intern(obj.data(), obj.size());
                rid = S.pool.intern(rel.data(), rel.size());
            }
            (void)last_obj;
            (void)last_rel;
            uint8_t kind = r->subject_kind[i] ? 1 : 0;
            uint32_t sid = 0, sso = 0, ssr = 0;
            int32_t ssns = 0;
            if (kind) {
                if (!r->ss_namespace_id || !r->ss_object_off || !r->ss_relation_off)
                    throw Error(KETOGPU_EINVAL, "subject-set row without subject_set columns");
                ssns = r->ss_namespace_id[i];
                std::string_view so = col(r->ss_object_data, r->ss_object_off, i);
                std::string_view sr = col(r->ss_relation_data, r->ss_relation_off, i);
                sso = S.pool.intern(so.data(), so.size());
                ssr = S.pool.intern(sr.data(), sr.size());
            } else {
                if (!r->subject_id_off) throw Error(KETOGPU_EINVAL, "subject-id row without subject_id column");
                std::string_view si = col(r->subject_id_data, r->subject_id_off, i);
                sid = S.pool.intern(si.data(), si.size());
            }
            if (b->flags & KETOGPU_BUILD_SORT) {
                b->raw.push_back({r->namespace_id[i], ssns, oid, rid, sid, sso, ssr, kind, (uint64_t)b->raw.size()});
            } else {
                bool regroup = !b->open || b->cur.ns != r->namespace_id[i] || b->cur.obj != oid || b->cur.rel != rid;
                b->add(r->namespace_id[i], oid, rid, kind, sid, ssns, sso, ssr);
                if (regroup) {
                    b->cur_obj.assign(obj.data(), obj.size());
                    b->cur_rel.assign(rel.data(), rel.size());
                }
            }
        }
        return KETOGPU_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
}

int ketogpu_builder_finish(ketogpu_builder *b, ketogpu_snapshot **out) {
    std::unique_ptr<ketogpu_builder> owned(b);
    try {
        *out = nullptr;
        if (!b) throw Error(KETOGPU_EINVAL, "null builder");
        finish_snapshot(b);
        *out = reinterpret_cast<ketogpu_snapshot *>(b->s.release());
        return KETOGPU_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
}

void ketogpu_builder_free(ketogpu_builder *b) { delete b; }

// Write-path freshness (R14).  The next snapshot version is the
// base's rows with a TransactRelationTuples batch applied (relationtuples.go:271-278):
// inserted rows join their group after equal rows (commit_time is the last ORDER BY key,
// :215; InsertRelationTuple stamps time.Now(), :128-149), then every row matching a
// delete (namespace id, object, relation, subject) is removed, duplicates included
// (DeleteRelationTuples, :178-201).  The merge uses the base's row order (KETOGPU_ORDER_*,
// the order of KETOGPU_BUILD_SORT); a base whose rows are not in that order fails loudly
// (EINVAL) when the merged stream is not grouped.  O(rows) on the host: the new version is complete
// and immutable, and engines swap to it (keto_amd/freshness.py).
// The next version from the base's rows, a write batch and (namespaces != NULL) a new
// namespace configuration: ketogpu_snapshot_apply and ketogpu_snapshot_set_namespaces.
static int rebuild(const ketogpu_snapshot *basep, const ketogpu_row_batch *inserts, const ketogpu_row_batch *deletes,
                   const ketogpu_namespace *namespaces, size_t num_namespaces, ketogpu_snapshot **out) {
    try {
        if (!basep || !out) throw Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        const Snapshot &B = *reinterpret_cast<const Snapshot *>(basep);
        std::shared_lock<std::shared_mutex> rd(B.mu);
        std::vector<ketogpu_namespace> nss;
        if (namespaces)
            nss.assign(namespaces, namespaces + num_namespaces);
        else
            for (const Namespace &n : B.namespaces) nss.push_back(ketogpu_namespace{n.id, n.name.c_str()});
        ketogpu_build_opts opts{B.page_size, (B.nulls_last ? KETOGPU_ORDER_NULLS_LAST : 0u) |
                                                 (B.writable ? KETOGPU_BUILD_WRITABLE : 0u)};
        ketogpu_builder *raw_b = nullptr;
        int rc = ketogpu_builder_new(nss.data(), nss.size(), &opts, &raw_b);
        if (rc) return rc;
        std::unique_ptr<ketogpu_builder> b(raw_b);
        Snapshot &S = *b->s;
        for (size_t i = 1; i < B.pool.size(); i++) {  // same string ids as the base
            std::string_view x = B.pool.get((uint32_t)i);
            S.pool.intern(x.data(), x.size());
        }
        // the write batch as rows of the new pool (same parsing as builder_append)
        auto rows_of = [&](const ketogpu_row_batch *r, uint64_t seq0) {
            std::vector<TupleRow> v;
            if (!r || !r->n) return v;
            if (!r->namespace_id || !r->object_off || !r->relation_off || !r->subject_kind)
                throw Error(KETOGPU_EINVAL, "row batch misses a required column");
            for (size_t i = 0; i < r->n; i++) {
                std::string_view obj = col(r->object_data, r->object_off, i), rel = col(r->relation_data, r->relation_off, i);
                TupleRow t{r->namespace_id[i], 0, S.pool.intern(obj.data(), obj.size()),
                           S.pool.intern(rel.data(), rel.size()), 0, 0, 0, (uint8_t)(r->subject_kind[i] ? 1 : 0),
                           seq0 + i};
                if (t.kind) {
                    if (!r->ss_namespace_id || !r->ss_object_off || !r->ss_relation_off)
                        throw Error(KETOGPU_EINVAL, "subject-set row without subject_set columns");
                    std::string_view so = col(r->ss_object_data, r->ss_object_off, i);
                    std::string_view sr = col(r->ss_relation_data, r->ss_relation_off, i);
                    t.ss_ns = r->ss_namespace_id[i];
                    t.ss_obj = S.pool.intern(so.data(), so.size());
                    t.ss_rel = S.pool.intern(sr.data(), sr.size());
                } else {
                    if (!r->subject_id_off) throw Error(KETOGPU_EINVAL, "subject-id row without subject_id column");
                    std::string_view si = col(r->subject_id_data, r->subject_id_off, i);
                    t.sid = S.pool.intern(si.data(), si.size());
                }
                v.push_back(t);
            }
            return v;
        };
        SortCmp cmp{S.pool, S.nulls_last};
        std::vector<TupleRow> ins = rows_of(inserts, 1ull << 62), del = rows_of(deletes, 0);
        std::stable_sort(ins.begin(), ins.end(), cmp);
        for (auto &d : del) d.seq = 0;  // a delete matches every commit_time
        std::sort(del.begin(), del.end(), cmp);
        auto same = [](const TupleRow &a, const TupleRow &c) {
            return a.ns == c.ns && a.obj == c.obj && a.rel == c.rel && a.kind == c.kind &&
                   (a.kind ? (a.ss_ns == c.ss_ns && a.ss_obj == c.ss_obj && a.ss_rel == c.ss_rel) : a.sid == c.sid);
        };
        auto deleted = [&](TupleRow r) {
            r.seq = 0;
            auto it = std::lower_bound(del.begin(), del.end(), r, cmp);
            return it != del.end() && same(*it, r);
        };
        auto emit = [&](const TupleRow &r) {
            if (!deleted(r)) b->add(r.ns, r.obj, r.rel, r.kind, r.sid, r.ss_ns, r.ss_obj, r.ss_rel);
        };
        size_t ii = 0;
        uint64_t seq = 0;
        for (const Group &g : B.groups) {
            for (uint32_t k = 0; k < g.full_len; k++) {
                TupleRow r;
                if (g.first_bad < 0 || k < (uint32_t)g.first_bad) {
                    const uint32_t v = B.group_col[g.begin + k];
                    r = TupleRow{g.ns, 0, g.obj, g.rel, 0, 0, 0, B.node_kind[v], 0};
                    if (r.kind == KETOGPU_SUBJECT_SET) {
                        r.ss_ns = B.node_ns[v];
                        r.ss_obj = B.node_a[v];
                        r.ss_rel = B.node_b[v];
                    } else {
                        r.sid = B.node_a[v];
                    }
                } else {
                    r = B.tail_rows[g.tail + (k - (uint32_t)g.first_bad)];
                }
                r.seq = seq++;
                while (ii < ins.size() && cmp(ins[ii], r)) emit(ins[ii++]);
                emit(r);
            }
        }
        while (ii < ins.size()) emit(ins[ii++]);
        ketogpu_snapshot *o = nullptr;
        rc = ketogpu_builder_finish(b.release(), &o);
        if (rc) return rc;
        *out = o;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

int ketogpu_snapshot_apply(const ketogpu_snapshot *base, const ketogpu_row_batch *inserts,
                           const ketogpu_row_batch *deletes, ketogpu_snapshot **out) {
    return rebuild(base, inserts, deletes, nullptr, 0, out);
}

// Namespace-configuration reload (internal/driver/config/provider.go:87-110 resets the
// namespace manager on every change of KeyNamespaces): the same rows under the new
// configuration, so page poisoning (R7, relationtuples.go:43-80) and name resolution
// follow it — rows of a removed namespace id poison their pages, a re-added one heals them.
int ketogpu_snapshot_set_namespaces(const ketogpu_snapshot *base, const ketogpu_namespace *namespaces,
                                    size_t num_namespaces, ketogpu_snapshot **out) {
    if (num_namespaces && !namespaces) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    static const ketogpu_namespace none{0, ""};
    return rebuild(base, nullptr, nullptr, num_namespaces ? namespaces : &none, num_namespaces, out);
}

void ketogpu_snapshot_free(ketogpu_snapshot *s) { delete reinterpret_cast<Snapshot *>(s); }

int ketogpu_snapshot_stats_get(const ketogpu_snapshot *s, ketogpu_snapshot_stats *out) {
    if (!s || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const Snapshot &S = *reinterpret_cast<const Snapshot *>(s);
    std::shared_lock<std::shared_mutex> rd(S.mu);
    *out = S.stats;
    return KETOGPU_OK;
}

int ketogpu_snapshot_graph(const ketogpu_snapshot *sp, ketogpu_graph_view *out) {
    if (!sp || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
    out->num_nodes = s.N;
    out->num_expandable = s.Nx;
    out->num_interior = s.Ni;
    out->fint_off = s.fint_off.data();
    out->fint_col = s.fint_col.data();
    out->rev_off = s.rev_off.data();
    out->rev_col = s.rev_col.data();
    return KETOGPU_OK;
}

}  // extern "C"
