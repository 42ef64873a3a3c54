// snapshot_write.cpp — in-place writes on a writable snapshot: read-your-writes freshness
// (R14) at a cost set by the write, not by the graph.
//
// The reference's write path is TransactRelationTuples (internal/persistence/sql/
// relationtuples.go:271-278): InsertRelationTuple per row (:128-149, commit_time =
// time.Now(), so an inserted row sorts after equal rows, ORDER BY :215), then
// DeleteRelationTuples (:178-201, every matching row, duplicates included).  The next
// GetRelationTuples sees the new rows.  ketogpu_snapshot_apply restates that by rebuilding
// the snapshot from all rows (O(rows)); this file restates it on the rows a batch touches:
//   host   the touched groups get their new row lists appended to group_col / row_col and
//          their RowRefs re-pointed (expand, exact checks and resolution see the write);
//          new subjects take reserved node ids (the never-expanded class is the last id
//          range, so appending keeps the class order the kernels rely on);
//   device each touched forward row fint(g) and reverse row rev(s) is rewritten inside its
//          own capacity (rows were laid out with free slots, make_writable below) and
//          logged; engines replay the log at their next call (device_engine.hip: sync).
// Edge records carry the row position and capacity of the node they point at, and
// capacities never change between rebuilds, so no record outside a touched row changes.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <map>
#include <mutex>

#include "ketogpu_internal.hpp"

namespace ketogpu {

namespace {

constexpr uint32_t kReservedRowSlots = 4;  // reverse-row capacity of a reserved (new) node

inline uint64_t free_slots(uint64_t deg) { return 2 + deg / 8; }

}  // namespace

// Lay out the compact device rows with free slots (KETOGPU_BUILD_WRITABLE):
//   fint(v), v < Nx:   real interior successors | Df x (2 + d/8)
//   rev(u), u < Ni:    real interior preds | Dbi x (2 + di/8) | other preds | Dbo x (2 + do/8)
//   rev(u), u >= Ni:   real preds | Dbo x (2 + d/8)
//   rev(u), N <= u < n_cap (reserved ids): Dbo x 4
// Only the interior prefix of an interior node's reverse row is read through records
// (its length is the record's `deg`), so only those rows need two free regions.
void make_writable(Snapshot &S) {
    const uint32_t Ni = S.Ni, Nx = S.Nx, N = S.N;
    const uint64_t reserve = std::max<uint64_t>(1024, N / 8);
    if ((uint64_t)N + reserve >= (1ull << 31)) throw Error(KETOGPU_EINVAL, "writable snapshot: too many nodes");
    S.n_cap = (uint32_t)(N + reserve);
    auto placeholder = [&](uint32_t v) { return v == S.Df || v == S.Dbi || v == S.Dbo; };

    std::vector<uint64_t> fo((size_t)Nx + 1, 0);
    for (uint32_t v = 0; v < Nx; v++) {
        const uint64_t d = S.fint_off[v + 1] - S.fint_off[v];
        fo[v + 1] = fo[v] + d + (placeholder(v) ? 0 : free_slots(d));
    }
    std::vector<uint32_t> fc(fo[Nx], S.Df);
    for (uint32_t v = 0; v < Nx; v++)
        std::copy(S.fint_col.begin() + S.fint_off[v], S.fint_col.begin() + S.fint_off[v + 1], fc.begin() + fo[v]);

    std::vector<uint64_t> ro((size_t)S.n_cap + 1, 0);
    auto split = [&](uint32_t u) -> uint64_t {  // real interior predecessors of u
        const uint32_t *b = S.rev_col.data() + S.rev_off[u], *e = S.rev_col.data() + S.rev_off[u + 1];
        return (uint64_t)(std::lower_bound(b, e, Ni) - b);
    };
    for (uint32_t u = 0; u < S.n_cap; u++) {
        uint64_t cap = 0;
        if (u >= N) {
            cap = kReservedRowSlots;
        } else if (!placeholder(u)) {
            const uint64_t d = S.rev_off[u + 1] - S.rev_off[u];
            if (u < Ni) {
                const uint64_t di = split(u);
                cap = di + free_slots(di) + (d - di) + free_slots(d - di);
            } else {
                cap = d + free_slots(d);
            }
        }
        ro[u + 1] = ro[u] + cap;
    }
    std::vector<uint32_t> rc(ro[S.n_cap], S.Dbo);
    for (uint32_t u = 0; u < N; u++) {
        if (placeholder(u)) continue;
        const uint64_t b = S.rev_off[u], d = S.rev_off[u + 1] - b;
        if (u < Ni) {
            const uint64_t di = split(u), ifree = free_slots(di);
            std::copy(S.rev_col.begin() + b, S.rev_col.begin() + b + di, rc.begin() + ro[u]);
            std::fill(rc.begin() + ro[u] + di, rc.begin() + ro[u] + di + ifree, S.Dbi);
            std::copy(S.rev_col.begin() + b + di, S.rev_col.begin() + b + d, rc.begin() + ro[u] + di + ifree);
        } else {
            std::copy(S.rev_col.begin() + b, S.rev_col.begin() + b + d, rc.begin() + ro[u]);
        }
    }
    S.fint_off.swap(fo);
    S.fint_col.swap(fc);
    S.rev_off.swap(ro);
    S.rev_col.swap(rc);
    index_groups(S);
    // room for the writes: new nodes take reserved ids, grown groups are appended
    for (auto *v : {&S.node_a, &S.node_b, &S.key_id}) v->reserve(S.n_cap);
    S.node_kind.reserve(S.n_cap);
    S.ambiguous.reserve(S.n_cap);
    S.node_ns.reserve(S.n_cap);
    S.node_row.reserve(S.n_cap);
    S.sid_node.reserve(S.sid_node.size() + reserve);
    S.group_col.reserve(S.group_col.size() + S.group_col.size() / 4 + 1024);
    S.row_col.reserve(S.row_col.size() + S.row_col.size() / 4 + 1024);
}

void index_groups(Snapshot &S) {
    S.group_idx = TripleMap();
    for (uint32_t gi = 0; gi < S.groups.size(); gi++) {
        const Group &g = S.groups[gi];
        S.group_idx.get_or_insert(g.ns, g.obj, g.rel, gi);
    }
}

namespace {

// A row's subject in ORDER BY terms (relationtuples.go:215): subject_id, or
// (subject_set_namespace_id, subject_set_object, subject_set_relation); subject-set rows
// have a NULL subject_id, which sorts first (SQLite) or last (Postgres, nulls_last).
struct SubjKey {
    uint8_t kind;
    int32_t ns;
    std::string_view a, b;
};

int cmp_bytes(std::string_view x, std::string_view y) {
    const int c = memcmp(x.data(), y.data(), std::min(x.size(), y.size()));
    if (c) return c;
    return x.size() < y.size() ? -1 : (x.size() > y.size());
}

int cmp_subj(const SubjKey &x, const SubjKey &y, bool nulls_last) {
    if (x.kind != y.kind) {
        const bool x_first = (x.kind == KETOGPU_SUBJECT_SET) != nulls_last;
        return x_first ? -1 : 1;
    }
    if (x.kind == KETOGPU_SUBJECT_ID) return cmp_bytes(x.a, y.a);
    if (x.ns != y.ns) return x.ns < y.ns ? -1 : 1;
    const int c = cmp_bytes(x.a, y.a);
    return c ? c : cmp_bytes(x.b, y.b);
}

inline std::string_view col(const char *data, const uint64_t *off, size_t i) {
    if (!data || !off) return std::string_view();
    return std::string_view(data + off[i], off[i + 1] - off[i]);
}

struct InRow {
    int32_t ns;
    std::string_view obj, rel;
    SubjKey subj;
    size_t seq;
};

std::vector<InRow> read_rows(const ketogpu_row_batch *r) {
    std::vector<InRow> v;
    if (!r || !r->n) return v;
    if (!r->namespace_id || !r->object_off || !r->relation_off || !r->subject_kind)
        throw Error(KETOGPU_EINVAL, "row batch misses a required column");
    for (size_t i = 0; i < r->n; i++) {
        InRow x{r->namespace_id[i], col(r->object_data, r->object_off, i), col(r->relation_data, r->relation_off, i),
                SubjKey{}, i};
        if (r->subject_kind[i]) {
            if (!r->ss_namespace_id || !r->ss_object_off || !r->ss_relation_off)
                throw Error(KETOGPU_EINVAL, "subject-set row without subject_set columns");
            x.subj = SubjKey{KETOGPU_SUBJECT_SET, r->ss_namespace_id[i], col(r->ss_object_data, r->ss_object_off, i),
                             col(r->ss_relation_data, r->ss_relation_off, i)};
        } else {
            if (!r->subject_id_off) throw Error(KETOGPU_EINVAL, "subject-id row without subject_id column");
            x.subj = SubjKey{KETOGPU_SUBJECT_ID, 0, col(r->subject_id_data, r->subject_id_off, i), {}};
        }
        v.push_back(x);
    }
    return v;
}

struct Refuse {
    int reason;
};

// One write batch, planned without touching the snapshot, then committed.
struct Writer {
    Snapshot &S;
    explicit Writer(Snapshot &s) : S(s) {}

    // subjects: an existing node id, or kNew + index into fresh (ids N + index on commit)
    static constexpr uint32_t kNew = 0x80000000u;
    struct Fresh {
        SubjKey key;
        std::string key_string;  // Subject.String() when it must be interned (R4)
    };
    std::vector<Fresh> fresh;
    std::map<std::string, uint32_t> fresh_by_key;  // typed identity -> fresh index

    struct GroupOps {
        std::vector<std::pair<SubjKey, uint32_t>> ins;  // (key, subject) in batch order
        std::vector<uint32_t> del;                     // subjects whose rows go
    };
    std::map<uint32_t, GroupOps> ops;  // group index -> ops
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> new_rows;  // group -> subjects

    uint64_t n_ins = 0, n_del = 0;

    SubjKey key_of(uint32_t s) const {
        if (s & kNew) return fresh[s & ~kNew].key;
        return SubjKey{S.node_kind[s], S.node_ns[s], S.pool.get(S.node_a[s]),
                       S.node_kind[s] == KETOGPU_SUBJECT_SET ? S.pool.get(S.node_b[s]) : std::string_view()};
    }
    bool ns_known(int32_t id) const { return S.ns_by_id(id) != nullptr; }

    static std::string typed(const SubjKey &k) {
        std::string t(1, (char)k.kind);
        t.append((const char *)&k.ns, sizeof k.ns);
        const uint32_t la = (uint32_t)k.a.size();
        t.append((const char *)&la, sizeof la);
        t.append(k.a);
        t.append(k.b);
        return t;
    }

    // existing node of a subject, NONE if it has none
    uint32_t find_node(const SubjKey &k) const {
        if (k.kind == KETOGPU_SUBJECT_ID) {
            const uint32_t sid = S.pool.find(k.a);
            return sid != NONE && sid < S.sid_node.size() ? S.sid_node[sid] : NONE;
        }
        const uint32_t o = S.pool.find(k.a), r = S.pool.find(k.b);
        return o == NONE || r == NONE ? NONE : S.set_node.get(k.ns, o, r);
    }

    // the subject of an inserted row: its node, or a fresh one (class "never expanded")
    uint32_t subject(const SubjKey &k) {
        const uint32_t v = find_node(k);
        if (v != NONE) {
            // an expandable node that becomes a subject becomes interior: a class change
            if (k.kind == KETOGPU_SUBJECT_SET && v >= S.Ni && v < S.Nx) throw Refuse{KETOGPU_WRITE_CLASS};
            return v;
        }
        const std::string t = typed(k);
        auto it = fresh_by_key.find(t);
        if (it != fresh_by_key.end()) return kNew | it->second;
        Fresh f{k, {}};
        // Subject.String() (definitions.go:164-170) of the new node must not be shared (R4)
        const bool need_key = k.kind == KETOGPU_SUBJECT_SET ||
                              (k.a.find(':') != std::string_view::npos && k.a.find('#') != std::string_view::npos);
        if (need_key) {
            if (k.kind == KETOGPU_SUBJECT_SET) {
                const Namespace *n = S.ns_by_id(k.ns);
                f.key_string = (n ? n->name : std::string()) + ":" + std::string(k.a) + "#" + std::string(k.b);
            } else {
                f.key_string = std::string(k.a);
            }
            if (S.key_pool.find(f.key_string) != NONE) throw Refuse{KETOGPU_WRITE_AMBIGUOUS};
            for (const Fresh &o : fresh)
                if (!o.key_string.empty() && o.key_string == f.key_string) throw Refuse{KETOGPU_WRITE_AMBIGUOUS};
        }
        if ((uint64_t)S.N + fresh.size() + 1 > S.n_cap) throw Refuse{KETOGPU_WRITE_RESERVE};
        fresh.push_back(std::move(f));
        fresh_by_key.emplace(t, (uint32_t)fresh.size() - 1);
        return kNew | (uint32_t)(fresh.size() - 1);
    }

    // the group of a row (NONE: no such group)
    uint32_t group_of(const InRow &r) const {
        const uint32_t o = S.pool.find(r.obj), rl = S.pool.find(r.rel);
        if (o == NONE || rl == NONE) return NONE;
        return S.group_idx.get(r.ns, o, rl);
    }

    void plan(const std::vector<InRow> &ins, const std::vector<InRow> &del) {
        if (S.stats.num_wildcard_nodes) throw Refuse{KETOGPU_WRITE_WILDCARD};
        if (S.has_ambiguous) throw Refuse{KETOGPU_WRITE_AMBIGUOUS};
        auto wildcard = [&](const SubjKey &k) {
            if (k.kind != KETOGPU_SUBJECT_SET) return false;
            const Namespace *n = S.ns_by_id(k.ns);
            return (n && n->name.empty()) || k.a.empty() || k.b.empty();
        };
        for (const InRow &r : ins) {
            if (!ns_known(r.ns) || (r.subj.kind == KETOGPU_SUBJECT_SET && !ns_known(r.subj.ns)))
                throw Refuse{KETOGPU_WRITE_POISON};  // toInternal fails on such rows (relationtuples.go:48-67)
            if (wildcard(r.subj)) throw Refuse{KETOGPU_WRITE_WILDCARD};
            const uint32_t gi = group_of(r);
            if (gi == NONE) throw Refuse{KETOGPU_WRITE_CLASS};  // a new group: a new expandable node
            const Group &g = S.groups[gi];
            if (g.first_bad >= 0) throw Refuse{KETOGPU_WRITE_POISON};
            const uint32_t v = S.set_node.get(g.ns, g.obj, g.rel);
            if (v == NONE || v >= S.Nx) throw Refuse{KETOGPU_WRITE_CLASS};
            ops[gi].ins.push_back({r.subj, subject(r.subj)});
            n_ins++;
        }
        for (const InRow &r : del) {
            const uint32_t gi = group_of(r);
            if (gi == NONE) continue;  // no such rows
            if (S.groups[gi].first_bad >= 0) throw Refuse{KETOGPU_WRITE_POISON};
            uint32_t s = find_node(r.subj);
            if (s == NONE) {  // maybe a subject this batch inserts
                auto it = fresh_by_key.find(typed(r.subj));
                if (it == fresh_by_key.end()) continue;
                s = kNew | it->second;
            }
            ops[gi].del.push_back(s);
        }
    }

    // new row lists of the touched groups (subjects, DB order).  An insert goes after the
    // last old row that sorts before or equal to it (binary search: the group's rows are
    // in ORDER BY order), deletes filter node ids; O(group rows) copying, O(log) compares.
    void merge() {
        for (auto &[gi, op] : ops) {
            const Group &g = S.groups[gi];
            const uint32_t *old = S.group_col.data() + g.begin;
            std::stable_sort(op.ins.begin(), op.ins.end(), [&](const auto &x, const auto &y) {
                return cmp_subj(x.first, y.first, S.nulls_last) < 0;
            });
            std::vector<uint32_t> out;
            out.reserve(g.valid + op.ins.size());
            uint32_t done = 0;
            for (const auto &[key, subj] : op.ins) {
                uint32_t lo = done, hi = g.valid;  // first old row that sorts after the insert
                while (lo < hi) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    if (cmp_subj(key_of(old[mid]), key, S.nulls_last) <= 0)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                out.insert(out.end(), old + done, old + lo);
                out.push_back(subj);
                done = lo;
            }
            out.insert(out.end(), old + done, old + g.valid);
            if (!op.del.empty()) {
                std::vector<uint32_t> &dl = op.del;
                std::sort(dl.begin(), dl.end());
                dl.erase(std::unique(dl.begin(), dl.end()), dl.end());
                const size_t before = out.size();
                if (dl.size() <= 8)  // a few deleted subjects: compare each row with all of them
                    out.erase(std::remove_if(out.begin(), out.end(),
                                             [&dl](uint32_t s) {
                                                 bool hit = false;
                                                 for (uint32_t d : dl) hit |= s == d;
                                                 return hit;
                                             }),
                              out.end());
                else
                    out.erase(std::remove_if(out.begin(), out.end(),
                                             [&dl](uint32_t s) { return std::binary_search(dl.begin(), dl.end(), s); }),
                              out.end());
                n_del += before - out.size();
            }
            new_rows.push_back({gi, std::move(out)});
        }
    }

    // grown groups are copied to the end of the row arrays; once the stale copies would
    // outweigh the live rows, the batch goes to the rebuild (which compacts)
    static uint32_t room(const Group &g) { return std::max(g.valid, g.cap); }
    void budget() const {
        uint64_t grow = 0;
        for (const auto &[gi, rows] : new_rows)
            if (rows.size() > room(S.groups[gi])) grow += room(S.groups[gi]);
        if (S.row_garbage + grow > std::max<uint64_t>(S.stats.num_edges, 1u << 20)) throw Refuse{KETOGPU_WRITE_FULL};
    }

    // device row edits: node -> (added, removed) neighbours
    struct RowEdit {
        std::vector<uint32_t> add, rem;
    };
    std::map<uint32_t, RowEdit> fwd, rev;  // fint(g) edits, rev(s) edits

    // edges that appear or disappear: only the batch's subjects can change.  Edge g -> s
    // existed iff g is in the (sorted) reverse row of s; afterwards it exists iff s was
    // inserted or was there, and was not deleted (a delete removes every duplicate)
    void diff() {
        for (auto &[gi, rows] : new_rows) {
            const Group &g = S.groups[gi];
            const uint32_t v = S.set_node.get(g.ns, g.obj, g.rel);
            const GroupOps &op = ops[gi];
            std::vector<uint32_t> ins_s, cand;
            for (const auto &x : op.ins) ins_s.push_back(x.second);
            std::sort(ins_s.begin(), ins_s.end());
            cand = ins_s;
            cand.insert(cand.end(), op.del.begin(), op.del.end());
            std::sort(cand.begin(), cand.end());
            cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
            for (uint32_t s : cand) {
                bool before = false;
                if (!(s & kNew)) {
                    const uint32_t *b = S.rev_col.data() + S.rev_off[s], *e = S.rev_col.data() + S.rev_off[s + 1];
                    before = std::binary_search(b, e, v);
                }
                const bool deleted = std::binary_search(op.del.begin(), op.del.end(), s);  // sorted in merge()
                const bool after = !deleted && (before || std::binary_search(ins_s.begin(), ins_s.end(), s));
                if (before == after) continue;
                const bool interior = !(s & kNew) && s < S.Ni;
                if (after) {
                    if (interior) fwd[v].add.push_back(s);
                    rev[s].add.push_back(v);
                } else {
                    if (interior) fwd[v].rem.push_back(s);
                    rev[s].rem.push_back(v);
                }
            }
        }
    }

    // final content of one device row region [b, e) whose free slots hold `pad`; the real
    // entries are the sorted prefix below `pad`
    static bool rewrite(std::vector<uint32_t> &col, uint64_t b, uint64_t e, uint32_t pad, std::vector<uint32_t> add,
                        std::vector<uint32_t> rem, bool commit, size_t *real_after = nullptr) {
        std::vector<uint32_t> cur;
        for (uint64_t i = b; i < e && col[i] != pad; i++) cur.push_back(col[i]);
        std::sort(add.begin(), add.end());
        std::sort(rem.begin(), rem.end());
        std::vector<uint32_t> tmp, out;
        std::set_difference(cur.begin(), cur.end(), rem.begin(), rem.end(), std::back_inserter(tmp));
        std::set_union(tmp.begin(), tmp.end(), add.begin(), add.end(), std::back_inserter(out));
        if (real_after) *real_after = out.size();
        if (out.size() > e - b) return false;
        if (commit) {
            std::copy(out.begin(), out.end(), col.begin() + b);
            std::fill(col.begin() + b + out.size(), col.begin() + e, pad);
        }
        return true;
    }

    // real entries of a row region (the sorted prefix below the placeholder)
    uint32_t real(const std::vector<uint32_t> &col, uint64_t b, uint64_t e, uint32_t pad) const {
        return (uint32_t)(std::lower_bound(col.begin() + b, col.begin() + e, pad) - (col.begin() + b));
    }
    std::vector<uint32_t> fcount_changed, icount_changed;  // nodes whose record fields changed

    // Rows re-uploaded because a record's count field changed (commit's second pass): one
    // nested-group insert into a hub group would re-upload the forward row of every one of
    // its (millions of) predecessors, so past this budget the write is refused
    // (KETOGPU_WRITE_FANOUT) and VersionedEngine rebuilds instead.
    static uint64_t fanout_budget() {
        const char *v = getenv("KETOGPU_WRITE_FANOUT_MAX");
        return v ? strtoull(v, nullptr, 10) : (uint64_t)1 << 16;
    }

    // check (commit = false) or apply (commit = true) the device row edits
    uint64_t device(bool commit) {
        auto id = [&](uint32_t s) { return (s & kNew) ? S.N + (s & ~kNew) : s; };
        uint64_t rows = 0, fanout = 0;
        for (auto &[v, ed] : fwd) {
            const uint32_t before = real(S.fint_col, S.fint_off[v], S.fint_off[v + 1], S.Df);
            size_t after = 0;
            if (!rewrite(S.fint_col, S.fint_off[v], S.fint_off[v + 1], S.Df, ed.add, ed.rem, commit, &after))
                throw Refuse{KETOGPU_WRITE_FULL};
            // only an interior node is pointed at by forward records
            if (v < S.Ni && after != before) {
                fanout += S.rev_off[v + 1] - S.rev_off[v];
                if (commit) fcount_changed.push_back(v);
            }
            if (commit) S.patches.push_back({0, v});
            rows++;
        }
        for (auto &[s0, ed] : rev) {
            const uint32_t u = id(s0);
            const uint64_t b = S.rev_off[u], e = S.rev_off[u + 1];
            std::vector<uint32_t> ai, ao, ri, ro;
            for (uint32_t x : ed.add) (x < S.Ni ? ai : ao).push_back(x);
            for (uint32_t x : ed.rem) (x < S.Ni ? ri : ro).push_back(x);
            bool ok;
            if (u < S.Ni) {  // interior part [b, m) padded with Dbi, then the other part
                uint64_t m = b;
                while (m < e && S.rev_col[m] < S.Ni) m++;
                const uint32_t before = real(S.rev_col, b, m, S.Dbi);
                size_t after = 0;
                ok = rewrite(S.rev_col, b, m, S.Dbi, ai, ri, commit, &after) &&
                     rewrite(S.rev_col, m, e, S.Dbo, ao, ro, commit);
                if (ok && after != before) {
                    fanout += S.node_row[u].len;
                    if (commit) icount_changed.push_back(u);
                }
            } else {
                std::vector<uint32_t> add(ai), rem(ri);
                add.insert(add.end(), ao.begin(), ao.end());
                rem.insert(rem.end(), ro.begin(), ro.end());
                ok = rewrite(S.rev_col, b, e, S.Dbo, add, rem, commit);
            }
            if (!ok) throw Refuse{KETOGPU_WRITE_FULL};
            if (commit) S.patches.push_back({1, u});
            rows++;
        }
        if (!commit && fanout > fanout_budget()) throw Refuse{KETOGPU_WRITE_FANOUT};
        return rows;
    }

    void commit(ketogpu_write_result &res) {
        // new subjects: reserved ids N, N+1, ... (never-expanded class, the last id range)
        for (Fresh &f : fresh) {
            const uint32_t v = S.N++;
            if (f.key.kind == KETOGPU_SUBJECT_ID) {
                const uint32_t sid = S.pool.intern(f.key.a.data(), f.key.a.size());
                if (S.sid_node.size() <= sid) S.sid_node.resize(sid + 1, NONE);  // capacity reserved
                S.sid_node[sid] = v;
                S.node_kind.push_back(KETOGPU_SUBJECT_ID);
                S.node_ns.push_back(0);
                S.node_a.push_back(sid);
                S.node_b.push_back(0);
            } else {
                const uint32_t o = S.pool.intern(f.key.a.data(), f.key.a.size());
                const uint32_t r = S.pool.intern(f.key.b.data(), f.key.b.size());
                S.set_node.get_or_insert(f.key.ns, o, r, v);
                S.node_kind.push_back(KETOGPU_SUBJECT_SET);
                S.node_ns.push_back(f.key.ns);
                S.node_a.push_back(o);
                S.node_b.push_back(r);
            }
            S.key_id.push_back(f.key_string.empty() ? (0x80000000u | v)
                                                    : S.key_pool.intern(f.key_string.data(), f.key_string.size()));
            S.ambiguous.push_back(0);
            S.node_row.push_back(RowRef{});
        }
        const uint32_t N0 = S.N - (uint32_t)fresh.size();
        auto id = [&](uint32_t s) { return (s & kNew) ? N0 + (s & ~kNew) : s; };
        // device rows first (they index new nodes by id), then the host rows
        const uint32_t Nsave = S.N;
        S.N = N0;  // device() maps fresh subjects through S.N
        res.device_rows = device(true);
        S.N = Nsave;
        uint64_t edges_delta = 0, edges_minus = 0;
        for (auto &[gi, rows] : new_rows) {
            Group &g = S.groups[gi];
            const uint32_t v = S.set_node.get(g.ns, g.obj, g.rel);
            edges_minus += g.valid;
            edges_delta += rows.size();
            RowRef rr = S.node_row[v];
            if (rows.size() > room(g)) {  // outgrown: a new copy with a quarter free at the end
                S.row_garbage += room(g);
                const uint64_t cap = rows.size() + rows.size() / 4 + 4;
                g.cap = (uint32_t)std::min<uint64_t>(cap, 0xffffffffu);
                g.begin = S.group_col.size();
                rr.off = S.row_col.size();
                S.group_col.resize(S.group_col.size() + g.cap);
                S.row_col.resize(S.row_col.size() + g.cap);
            }
            for (size_t k = 0; k < rows.size(); k++) S.group_col[g.begin + k] = S.row_col[rr.off + k] = id(rows[k]);
            rr.len = rr.full_len = (uint32_t)rows.size();
            rr.first_bad = -1;
            g.valid = g.full_len = (uint32_t)rows.size();
            S.node_row[v] = rr;
        }
        // Edge records carry the real entry counts of the rows they point at (the free slots
        // are never read through a record): rows holding a record for a node whose count
        // changed are re-uploaded too — fint(p) for each (expandable) predecessor p of an
        // interior node whose interior successors changed, rev(x) for each successor x of an
        // interior node whose interior predecessors changed
        for (uint32_t v : fcount_changed)  // every expandable predecessor (fint rows of all of them)
            for (uint64_t k = S.rev_off[v]; k < S.rev_off[v + 1]; k++) {
                const uint32_t p = S.rev_col[k];
                if (p != S.Dbi && p != S.Dbo) S.patches.push_back({0, p}), res.device_rows++;
            }
        for (uint32_t u : icount_changed) {
            const RowRef &r = S.node_row[u];
            std::vector<uint32_t> xs(S.row_col.begin() + r.off, S.row_col.begin() + r.off + r.len);
            std::sort(xs.begin(), xs.end());
            xs.erase(std::unique(xs.begin(), xs.end()), xs.end());
            for (uint32_t x : xs) S.patches.push_back({1, x}), res.device_rows++;
        }
        auto &st = S.stats;
        st.num_rows = st.num_rows + n_ins - n_del;
        st.num_edges = st.num_edges + edges_delta - edges_minus;
        st.num_nodes = S.N;
        for (auto &[v, ed] : fwd) st.num_interior_edges += ed.add.size() - ed.rem.size();
        for (auto &[s, ed] : rev) st.num_rev_edges += ed.add.size() - ed.rem.size();
        S.version++;
        S.trim_patches();  // the log keeps only what some engine has not replayed yet
        res.applied = 1;
        res.reason = KETOGPU_WRITE_APPLIED;
        res.rows_inserted = n_ins;
        res.rows_deleted = n_del;
        res.groups_touched = new_rows.size();
        res.new_nodes = fresh.size();
    }
};

}  // namespace
}  // namespace ketogpu

using namespace ketogpu;

extern "C" {

int ketogpu_snapshot_write(ketogpu_snapshot *sp, const ketogpu_row_batch *inserts, const ketogpu_row_batch *deletes,
                           ketogpu_write_result *res) {
    try {
        if (!sp || !res) throw Error(KETOGPU_EINVAL, "null argument");
        const auto t0 = std::chrono::steady_clock::now();
        *res = ketogpu_write_result{};
        Snapshot &S = *reinterpret_cast<Snapshot *>(sp);
        const std::vector<InRow> ins = read_rows(inserts), del = read_rows(deletes);
        std::unique_lock<std::shared_mutex> wr(S.mu);
        res->version = S.version;
        if (!S.writable) {
            res->reason = KETOGPU_WRITE_NOT_WRITABLE;
        } else {
            Writer w(S);
            try {
                w.plan(ins, del);
                w.merge();
                w.budget();
                w.diff();
                w.device(false);  // every touched row fits: nothing below can refuse
            } catch (const Refuse &r) {
                res->reason = r.reason;
            }
            if (!res->reason) w.commit(*res);
            res->version = S.version;
        }
        res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

uint64_t ketogpu_snapshot_version(const ketogpu_snapshot *sp) {
    if (!sp) return 0;
    const Snapshot &S = *reinterpret_cast<const Snapshot *>(sp);
    std::shared_lock<std::shared_mutex> rd(S.mu);
    return S.version;
}

}  // extern "C"
