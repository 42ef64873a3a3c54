// host_engine.cpp — request resolution and the sequential (order-dependent) engine
// paths over the snapshot:
//   * resolve_root / resolve_subject: strings -> node ids (namespace by first match,
//     internal/driver/config/namespace_memory.go:29-47; typed equality,
//     internal/relationtuple/definitions.go:253-267),
//   * exact_check: the reference's DFS with its Subject.String()-keyed visited set and
//     per-root-tuple fresh maps (internal/check/engine.go:33-95,
//     internal/x/graph/graph_utils.go:13-35); used only for requests the GPU flags as
//     touching an ambiguous key (R4), where the sequential order decides the answer,
//   * BuildTree (internal/expand/engine.go:30-98): sequential DFS over the ordered rows;
//     its output order depends on DB order, so it stays a host walk of the snapshot.
#include <string>
#include <unordered_set>

#include "ketogpu_internal.hpp"

namespace ketogpu {

static thread_local std::string g_last_error;
void set_last_error(const std::string &msg) { g_last_error = msg; }

static inline const char *nz(const char *p) { return p ? p : ""; }

ResolvedRoot resolve_root(const Snapshot &s, std::string_view ns, std::string_view obj, std::string_view rel) {
    ResolvedRoot r;
    r.any_ns = ns.empty();
    r.any_obj = obj.empty();
    r.any_rel = rel.empty();
    if (!r.any_ns) {
        const Namespace *n = s.ns_by_name(ns);
        if (!n) {  // GetNamespaceByName -> herodot.ErrNotFound (relationtuples.go:230-236)
            r.kind = ResolvedRoot::UNKNOWN_NS;
            return r;
        }
        r.ns = n->id;
    }
    uint32_t oid = r.any_obj ? 0 : s.pool.find(obj), rid = r.any_rel ? 0 : s.pool.find(rel);
    if (oid == NONE || rid == NONE) {  // a string no tuple has: the query returns nothing
        r.kind = ResolvedRoot::EMPTY;
        return r;
    }
    r.obj = oid;
    r.rel = rid;
    // The request is the query of the subject set (ns, obj, rel); a snapshot node with
    // that identity has exactly this query's rows.  For ns == "" only the namespace
    // named "" (if configured) gives a node whose query is namespace-agnostic.
    bool have_ns_node = !r.any_ns || s.has_empty_name_ns;
    int32_t node_ns = r.any_ns ? s.empty_name_ns : r.ns;
    if (have_ns_node) {
        uint32_t v = s.set_node.get(node_ns, oid, rid);
        if (v != NONE) {
            if (s.node_row[v].len) {
                r.kind = ResolvedRoot::NODE;
                r.node = v;
            } else {
                r.kind = ResolvedRoot::EMPTY;
            }
            return r;
        }
    }
    if (!r.any_ns && !r.any_obj && !r.any_rel) {
        r.kind = ResolvedRoot::EMPTY;  // a concrete group that does not exist
        return r;
    }
    r.kind = ResolvedRoot::DYNAMIC;
    return r;
}

uint32_t resolve_subject(const Snapshot &s, int kind, std::string_view id, std::string_view ns, std::string_view obj,
                         std::string_view rel) {
    if (kind == KETOGPU_SUBJECT_ID) {
        uint32_t sid = s.pool.find(id);
        if (sid == NONE || sid >= s.sid_node.size()) return NONE;
        return s.sid_node[sid];
    }
    if (kind == KETOGPU_SUBJECT_SET) {
        // reached subject sets carry the configured name of their namespace id
        // (relationtuples.go:64-76): a name that is not configured never matches
        const Namespace *n = s.ns_by_name(ns);
        if (!n) return NONE;
        uint32_t o = s.pool.find(obj), r = s.pool.find(rel);
        if (o == NONE || r == NONE) return NONE;
        return s.set_node.get(n->id, o, r);
    }
    return NONE;
}

uint32_t resolve_subject(const Snapshot &s, const ketogpu_subject &subj) {
    return resolve_subject(s, subj.kind, sv(subj.id), sv(subj.ns), sv(subj.obj), sv(subj.rel));
}

// The reference DFS, iterative (explicit stack) so deep graphs cannot overflow the
// caller's (cgo) thread stack.  Visiting order is exactly the recursive order: rows of a
// query in DB order, the subtree of a subject set before the next row.
bool exact_check(const Snapshot &s, const uint32_t *root_rows, uint32_t root_len, const ketogpu_subject &,
                 uint32_t target) {
    if (target == NONE) return false;
    struct Frame {
        const uint32_t *p;
        uint32_t n, i;
    };
    std::vector<Frame> st;
    std::unordered_set<uint32_t> visited;
    for (uint32_t i = 0; i < root_len; i++) {
        // top level: CheckAndAddVisited creates a fresh map for every root tuple
        // (engine.go:40 shadows ctx inside the loop; graph_utils.go:14-19)
        uint32_t u = root_rows[i];
        visited.clear();
        visited.insert(s.key_id[u]);
        if (u == target) return true;
        if (s.node_kind[u] != KETOGPU_SUBJECT_SET || !s.node_row[u].len) continue;
        st.clear();
        st.push_back({s.row_ptr(u), s.node_row[u].len, 0});
        while (!st.empty()) {
            Frame &f = st.back();
            if (f.i == f.n) {
                st.pop_back();
                continue;
            }
            uint32_t w = f.p[f.i++];
            if (!visited.insert(s.key_id[w]).second) continue;  // wasAlreadyVisited
            if (w == target) return true;                        // Equals (typed)
            if (s.node_kind[w] == KETOGPU_SUBJECT_SET && s.node_row[w].len)
                st.push_back({s.row_ptr(w), s.node_row[w].len, 0});
        }
    }
    return false;
}

}  // namespace ketogpu

using namespace ketogpu;

// -------------------------------------------------------------------- expand
struct ketogpu_tree {
    std::vector<ketogpu_tree_node> nodes;
    std::vector<std::unique_ptr<char[]>> strs;
    const char *dup(std::string_view v) {
        strs.emplace_back(new char[v.size() + 1]);
        memcpy(strs.back().get(), v.data(), v.size());
        strs.back()[v.size()] = 0;
        return strs.back().get();
    }
};

namespace {

struct TreeNode {
    int type;
    uint32_t node;                  // snapshot node, or NONE for a dynamic root
    std::vector<TreeNode> children;
};

struct Expander {
    const Snapshot &s;
    std::unordered_set<uint32_t> visited;  // one map for the whole tree (graph_utils.go)
    size_t ps;

    // returns false for nil; throws Error(ENOTFOUND) for a failing page
    bool build(uint32_t v, uint32_t key, const RowRef &q, const uint32_t *rows, int depth, TreeNode &out) {
        // engine.go:35-39: a subject set is marked visited before its rows are fetched
        if (!visited.insert(key).second) return false;
        out.type = KETOGPU_NODE_UNION;
        out.node = v;
        uint64_t total = q.full_len;
        for (uint64_t page = 0;; page++) {
            uint64_t b = page * ps, e = std::min<uint64_t>(b + ps, total);
            if (q.first_bad >= 0 && (uint64_t)q.first_bad < e)
                throw Error(KETOGPU_ENOTFOUND, "Unknown namespace id in a tuple of the expanded set");
            if (b >= e) return false;  // empty page (engine.go:64-65)
            if (depth <= 1) {          // engine.go:68-71
                out.type = KETOGPU_NODE_LEAF;
                return true;
            }
            for (uint64_t i = b; i < e; i++) {
                uint32_t u = rows[i];
                TreeNode c;
                if (!child(u, depth - 1, c)) c = TreeNode{KETOGPU_NODE_LEAF, u, {}};
                out.children.push_back(std::move(c));
            }
            if (e >= total) return true;
        }
    }

    bool child(uint32_t u, int depth, TreeNode &out) {
        if (depth <= 0) return false;
        if (s.node_kind[u] != KETOGPU_SUBJECT_SET) {
            out = TreeNode{KETOGPU_NODE_LEAF, u, {}};
            return true;
        }
        return build(u, s.key_id[u], s.node_row[u], s.row_ptr(u), depth, out);
    }
};

void fill_subject(const Snapshot &s, ketogpu_tree &t, uint32_t v, ketogpu_subject &out) {
    out.kind = s.node_kind[v];
    if (out.kind == KETOGPU_SUBJECT_ID) {
        out.id = t.dup(s.pool.get(s.node_a[v]));
        out.ns = out.obj = out.rel = nullptr;
    } else {
        const Namespace *n = s.ns_by_id(s.node_ns[v]);
        out.id = nullptr;
        out.ns = t.dup(n ? n->name : "");
        out.obj = t.dup(s.pool.get(s.node_a[v]));
        out.rel = t.dup(s.pool.get(s.node_b[v]));
    }
}

void flatten(const Snapshot &s, ketogpu_tree &t, const TreeNode &n, const ketogpu_subject &root_subj, bool is_root) {
    ketogpu_tree_node out{};
    out.type = n.type;
    out.num_children = (uint32_t)n.children.size();
    if (is_root && n.node == NONE) {
        out.subject.kind = root_subj.kind;
        out.subject.id = root_subj.kind == KETOGPU_SUBJECT_ID ? t.dup(nz(root_subj.id)) : nullptr;
        out.subject.ns = root_subj.kind == KETOGPU_SUBJECT_SET ? t.dup(nz(root_subj.ns)) : nullptr;
        out.subject.obj = root_subj.kind == KETOGPU_SUBJECT_SET ? t.dup(nz(root_subj.obj)) : nullptr;
        out.subject.rel = root_subj.kind == KETOGPU_SUBJECT_SET ? t.dup(nz(root_subj.rel)) : nullptr;
    } else {
        fill_subject(s, t, n.node, out.subject);
    }
    t.nodes.push_back(out);
    for (auto &c : n.children) flatten(s, t, c, root_subj, false);
}

void json_str(std::string &o, const char *p) {
    o += '"';
    for (const unsigned char *c = (const unsigned char *)nz(p); *c; c++) {
        if (*c == '"' || *c == '\\') {
            o += '\\';
            o += (char)*c;
        } else if (*c < 0x20) {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", *c);
            o += b;
        } else {
            o += (char)*c;
        }
    }
    o += '"';
}

size_t json_node(std::string &o, const ketogpu_tree &t, size_t i) {
    const ketogpu_tree_node &n = t.nodes[i];
    o += n.type == KETOGPU_NODE_UNION ? "{\"type\":\"union\"," : "{\"type\":\"leaf\",";
    size_t next = i + 1;
    if (n.num_children) {
        o += "\"children\":[";
        for (uint32_t c = 0; c < n.num_children; c++) {
            if (c) o += ',';
            next = json_node(o, t, next);
        }
        o += "],";
    }
    if (n.subject.kind == KETOGPU_SUBJECT_ID) {
        o += "\"subject_id\":";
        json_str(o, n.subject.id);
    } else {
        o += "\"subject_set\":{\"namespace\":";
        json_str(o, n.subject.ns);
        o += ",\"object\":";
        json_str(o, n.subject.obj);
        o += ",\"relation\":";
        json_str(o, n.subject.rel);
        o += '}';
    }
    o += '}';
    return next;
}

}  // namespace

extern "C" {

const char *ketogpu_last_error(void) { return g_last_error.c_str(); }
int ketogpu_abi_version(void) { return KETOGPU_ABI_VERSION; }
void ketogpu_free(void *p) { free(p); }

int ketogpu_resolve(const ketogpu_snapshot *sp, const ketogpu_check_request *req, uint32_t *root,
                    uint32_t *target) {
    if (!sp || !req || !root || !target) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
    std::shared_lock<std::shared_mutex> rd(s.mu);  // against in-place writes
    *root = NONE;
    *target = NONE;
    if (req->subject.kind != KETOGPU_SUBJECT_ID && req->subject.kind != KETOGPU_SUBJECT_SET) {
        set_last_error("subject is not allowed to be nil");  // relationtuple.ErrNilSubject
        return KETOGPU_EINVAL;
    }
    ResolvedRoot r = resolve_root(s, sv(req->ns), sv(req->obj), sv(req->rel));
    *target = resolve_subject(s, req->subject);
    if (r.kind == ResolvedRoot::NODE) *root = r.node;
    if (r.kind == ResolvedRoot::DYNAMIC) {
        set_last_error("wildcard root query without a snapshot node");
        return KETOGPU_ENOTFOUND;
    }
    return KETOGPU_OK;
}

int ketogpu_resolve_batch(const ketogpu_snapshot *sp, const ketogpu_request_batch *q, uint32_t *roots,
                          uint32_t *targets, int32_t *status) {
    if (!sp || !q || (q->n && (!roots || !targets || !q->ns_off || !q->obj_off || !q->rel_off))) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
    std::shared_lock<std::shared_mutex> rd(s.mu);  // against in-place writes
    auto col = [](const char *d, const uint64_t *o, size_t i) {
        return (d && o) ? std::string_view(d + o[i], o[i + 1] - o[i]) : std::string_view();
    };
    for (size_t i = 0; i < q->n; i++) {
        int kind = q->subject_kind ? (q->subject_kind[i] == 255 ? KETOGPU_SUBJECT_NIL : q->subject_kind[i])
                                   : KETOGPU_SUBJECT_ID;
        roots[i] = targets[i] = NONE;
        int32_t st = KETOGPU_OK;
        if (kind != KETOGPU_SUBJECT_ID && kind != KETOGPU_SUBJECT_SET) {
            st = KETOGPU_EINVAL;
        } else {
            ResolvedRoot r = resolve_root(s, col(q->ns_data, q->ns_off, i), col(q->obj_data, q->obj_off, i),
                                          col(q->rel_data, q->rel_off, i));
            targets[i] = resolve_subject(s, kind, col(q->sid_data, q->sid_off, i), col(q->ss_ns_data, q->ss_ns_off, i),
                                         col(q->ss_obj_data, q->ss_obj_off, i), col(q->ss_rel_data, q->ss_rel_off, i));
            if (r.kind == ResolvedRoot::NODE) roots[i] = r.node;
            if (r.kind == ResolvedRoot::DYNAMIC) st = KETOGPU_ENOTFOUND;
        }
        if (status) status[i] = st;
    }
    return KETOGPU_OK;
}

int ketogpu_expand(const ketogpu_snapshot *sp, const ketogpu_subject *subj, int32_t rest_depth,
                   ketogpu_tree **out) {
    try {
        if (!sp || !subj || !out) throw Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
        std::shared_lock<std::shared_mutex> rd(s.mu);  // against in-place writes
        if (subj->kind != KETOGPU_SUBJECT_ID && subj->kind != KETOGPU_SUBJECT_SET)
            throw Error(KETOGPU_EINVAL, "subject is not allowed to be nil");
        if (rest_depth <= 0) return KETOGPU_OK;  // engine.go:31-33
        Expander ex{s, {}, (size_t)s.page_size};
        TreeNode root;
        bool ok;
        if (subj->kind == KETOGPU_SUBJECT_ID) {
            root = TreeNode{KETOGPU_NODE_LEAF, resolve_subject(s, *subj), {}};  // engine.go:93-97
            ok = true;
        } else {
            uint32_t v = resolve_subject(s, *subj);
            if (v != NONE) {
                ok = ex.child(v, rest_depth, root);
            } else {
                // A subject set that is not a snapshot node: its query may still match rows
                // through empty-field wildcards, or fail on an unknown namespace.
                ResolvedRoot r = resolve_root(s, sv(subj->ns), sv(subj->obj), sv(subj->rel));
                if (r.kind == ResolvedRoot::UNKNOWN_NS)
                    throw Error(KETOGPU_ENOTFOUND, std::string("Unknown namespace with name ") + nz(subj->ns) + ".");
                std::vector<uint32_t> rows;
                RowRef q;
                if (r.kind == ResolvedRoot::DYNAMIC || r.kind == ResolvedRoot::NODE) {
                    q = s.materialize(r.any_ns, r.ns, r.obj, r.any_obj, r.rel, r.any_rel, rows);
                    q.off = 0;
                }
                // its key cannot collide with a node key (else resolve_subject found it)
                // except through ':'/'#' ambiguity: use the string to be exact
                std::string key = std::string(nz(subj->ns)) + ":" + nz(subj->obj) + "#" + nz(subj->rel);
                uint32_t kid = s.key_pool.find(key);
                if (kid == NONE) kid = 0x40000000u;  // no node has this key
                ok = ex.build(NONE, kid, q, rows.data(), rest_depth, root);
                if (ok) root.node = NONE;
            }
        }
        if (!ok) return KETOGPU_OK;  // nil tree
        auto t = std::make_unique<ketogpu_tree>();
        if (root.node == NONE && subj->kind == KETOGPU_SUBJECT_ID) {
            ketogpu_tree_node n{};
            n.type = KETOGPU_NODE_LEAF;
            n.subject.kind = KETOGPU_SUBJECT_ID;
            n.subject.id = t->dup(nz(subj->id));
            t->nodes.push_back(n);
        } else {
            flatten(s, *t, root, *subj, true);
        }
        *out = t.release();
        return KETOGPU_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
}

int ketogpu_tree_nodes(const ketogpu_tree *t, const ketogpu_tree_node **nodes, size_t *n) {
    if (!t || !nodes || !n) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    *nodes = t->nodes.data();
    *n = t->nodes.size();
    return KETOGPU_OK;
}

int ketogpu_tree_json(const ketogpu_tree *t, char **json) {
    if (!json) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    std::string o;
    if (!t || t->nodes.empty())
        o = "null";
    else
        json_node(o, *t, 0);
    *json = (char *)malloc(o.size() + 1);
    if (!*json) return KETOGPU_ENOMEM;
    memcpy(*json, o.c_str(), o.size() + 1);
    return KETOGPU_OK;
}

void ketogpu_tree_free(ketogpu_tree *t) { delete t; }

}  // extern "C"
