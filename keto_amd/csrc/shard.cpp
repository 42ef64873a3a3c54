// shard.cpp — partition-aware snapshot loader (BASELINE.json config #5; SURVEY.md 8(e)
// "Partitioned"): a graph too large for one GPU, or one host, is loaded by every rank
// from the ONE ordered row read the single-GPU loader uses
// (internal/persistence/sql/relationtuples.go:203-258, ORDER BY :215, nid filter
// persister.go:94-96), and each rank keeps only the part it owns.
//
// Ownership.  A node is a typed subject (internal/relationtuple/definitions.go:253-267):
// a subject set (namespace id, object, relation) — which is also the group of rows whose
// query it expands to — or a subject id.  Its identity is hashed (salted 64-bit hash of
// the typed key) and rank owner = hash % world keeps it.  While streaming, a rank keeps
//   * the rows of every group it owns (its forward rows), and
//   * every row whose subject it owns (its reverse rows: subject <- group),
// after the reference's page-poison truncation (rows with an unknown namespace id poison
// their page and every later one, relationtuples.go:43-80,248-255; R7), which every rank
// computes itself because it sees every group's rows in order.  Memory per rank is
// O(rows / world + nodes / world): no rank interns the whole graph.
//
// Node ids.  After the stream each owner numbers its nodes by class — interior
// (expandable and a subject), other expandable, never expanded — and the global id
// interleaves the ranks inside each class range:
//   class 0:  v = l * world + r               (Ni = world * max_r Nil_r)
//   class 1:  v = Ni + (l - Nil_r) * world + r (Nx = Ni + world * max_r (Nxl_r - Nil_r))
//   class 2:  v = Nx + (l - Nxl_r) * world + r
// so owner(v) and the owner's local index are arithmetic (no per-node tables), interior
// ids are still the smallest (sorted rows keep interior entries first), and the rows the
// device kernels read look exactly like the single-GPU snapshot's (partition.hip).
// The ids of the nodes a rank references but does not own come from one exchange of
// hashes with their owners (ketogpu_shard_queries / _answer / _apply; the caller moves the
// arrays with torch.distributed all_to_all).
//
// Checked, with every rank reaching the same verdict: a 64-bit hash collision between two
// owned nodes (KETOGPU_ECOLLISION: reload with another salt), groups that are not
// contiguous in the stream (rows not in ORDER BY order), wildcard subject sets (R5:
// their rows are the union of many groups, materialized only by the whole-graph loader)
// and Subject.String() keys shared by two nodes (R4, ketogpu_shard_claims /
// _check_claims): the partitioned engine refuses such graphs as before.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "ketogpu_internal.hpp"

using namespace ketogpu;

namespace {

inline std::string_view col(const char *data, const uint64_t *off, size_t i) {
    if (!data || !off) return std::string_view();
    return std::string_view(data + off[i], off[i + 1] - off[i]);
}

// salted 64-bit hash of a byte string (8-byte words through mix64; collisions between
// owned nodes are detected exactly, so only the spread matters)
inline uint64_t absorb(uint64_t h, const char *p, size_t n) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    return mix64(h ^ w ^ ((uint64_t)(n - i) << 56)) + 0x632be59bd9b4e019ull;
}

// typed keys: [kind][ns id][object length][object][relation] | [kind][subject id]
inline void key_set(std::string &k, int32_t ns, std::string_view obj, std::string_view rel) {
    k.clear();
    k.push_back('\1');
    k.append((const char *)&ns, 4);
    const uint32_t n = (uint32_t)obj.size();
    k.append((const char *)&n, 4);
    k.append(obj.data(), obj.size());
    k.append(rel.data(), rel.size());
}
inline void key_id(std::string &k, std::string_view sid) {
    k.clear();
    k.push_back('\0');
    k.append(sid.data(), sid.size());
}
// KETOGPU_SHARD_HASH_BITS (tests only) narrows node hashes so collisions actually happen
inline uint64_t hash_mask() {
    static const uint64_t m = [] {
        const char *e = getenv("KETOGPU_SHARD_HASH_BITS");
        const int b = e ? atoi(e) : 64;
        return b >= 64 || b <= 0 ? ~0ull : (1ull << b) - 1;
    }();
    return m;
}
inline uint64_t key_hash(uint64_t salt, const std::string &k) {
    return absorb(mix64(salt ^ 0x4b45544f53484152ull), k.data(), k.size()) & hash_mask();
}

// hash -> u32 (open addressing; hash 0 is remapped so 0 can mark empty slots)
class HashIndex {
  public:
    HashIndex() { rehash(1 << 10); }
    static uint64_t fix(uint64_t h) { return h ? h : 1; }
    uint32_t get(uint64_t h) const {
        h = fix(h);
        for (size_t i = slot(h);; i = (i + 1) & mask_) {
            if (keys_[i] == h) return vals_[i];
            if (!keys_[i]) return NONE;
        }
    }
    // value of h, inserting v when absent; `fresh` tells which
    uint32_t get_or_insert(uint64_t h, uint32_t v, bool &fresh) {
        if ((n_ + 1) * 4 > keys_.size() * 3) rehash(keys_.size() * 2);
        h = fix(h);
        for (size_t i = slot(h);; i = (i + 1) & mask_) {
            if (keys_[i] == h) {
                fresh = false;
                return vals_[i];
            }
            if (!keys_[i]) {
                keys_[i] = h;
                vals_[i] = v;
                n_++;
                fresh = true;
                return v;
            }
        }
    }
    void reserve(size_t n) {
        size_t c = keys_.size();
        while (n * 4 > c * 3) c *= 2;
        if (c != keys_.size()) rehash(c);
    }
    size_t bytes() const { return keys_.capacity() * 8 + vals_.capacity() * 4; }
    void clear() {
        std::vector<uint64_t>().swap(keys_);
        std::vector<uint32_t>().swap(vals_);
        n_ = 0;
        rehash(1 << 4);
    }

  private:
    // the slot from the hash's high bits: an owner keeps hashes with equal h % world, so
    // their low bits are alike (Fibonacci hashing spreads them)
    size_t slot(uint64_t h) const { return (size_t)((h * 0x9e3779b97f4a7c15ull) >> (64 - bits_)); }
    void rehash(size_t cap) {
        std::vector<uint64_t> ok;
        std::vector<uint32_t> ov;
        ok.swap(keys_);
        ov.swap(vals_);
        keys_.assign(cap, 0);
        vals_.assign(cap, NONE);
        mask_ = cap - 1;
        bits_ = 0;
        while ((size_t(1) << bits_) < cap) bits_++;
        n_ = 0;
        for (size_t i = 0; i < ok.size(); i++)
            if (ok[i]) {
                size_t j = slot(ok[i]);
                while (keys_[j]) j = (j + 1) & mask_;
                keys_[j] = ok[i];
                vals_[j] = ov[i];
                n_++;
            }
    }
    std::vector<uint64_t> keys_;
    std::vector<uint32_t> vals_;
    size_t n_ = 0, mask_ = 0;
    int bits_ = 0;
};

template <class T>
size_t vbytes(const std::vector<T> &v) {
    return v.capacity() * sizeof(T);
}

constexpr uint8_t kExp = 1, kSub = 2, kSet = 4, kClosed = 8;  // kClosed: an owned group's rows ended

}  // namespace

struct ketogpu_shard {
    // configuration (every rank alike)
    std::vector<Namespace> namespaces;
    int page_size = 100;
    uint32_t rank = 0, world = 1;
    uint64_t salt = 0;
    // owned nodes in registration order: hash, flags, typed key (collision check) and
    // Subject.String() key hash (R4 claims)
    std::vector<uint64_t> node_h, node_kh;
    std::vector<uint8_t> node_flags;
    std::vector<uint64_t> key_off;
    std::vector<char> keys;
    HashIndex index;  // hash -> registration index
    // forward rows of owned expandable groups: (registration index, [begin, end) of fcol)
    std::vector<uint32_t> frow_node;
    std::vector<uint64_t> frow_begin;
    std::vector<uint64_t> fcol;  // subject hashes, valid prefix only
    // reverse rows: (owned subject's registration index, group hash)
    std::vector<uint32_t> rsub;
    std::vector<uint64_t> rgrp;
    // local numbering (after finish): registration index -> local id; counts per class
    std::vector<uint32_t> local;
    uint64_t nil = 0, nxl = 0, nl = 0;
    // global layout (after set_layout)
    bool laid_out = false;
    uint64_t Ni = 0, Nx = 0, N = 0;
    // id exchange: distinct referenced hashes grouped by owner, their counts
    std::vector<uint64_t> q_hash;
    std::vector<uint64_t> q_count;
    // device rows (global ids), after apply
    bool ready = false;
    std::vector<uint64_t> lf_off, lr_off, lb_off;
    std::vector<uint32_t> lf_col, lr_col, lb_col;
    ketogpu_shard_stats stats{};

    uint32_t owner_of_hash(uint64_t h) const { return (uint32_t)(h % world); }
    uint64_t global_of_local(uint64_t l) const {
        const uint64_t W = world, r = rank;
        if (l < nil) return l * W + r;
        if (l < nxl) return Ni + (l - nil) * W + r;
        return Nx + (l - nxl) * W + r;
    }
    const Namespace *ns_by_id(int32_t id) const {
        for (auto &n : namespaces)
            if (n.id == id) return &n;
        return nullptr;
    }
    const Namespace *ns_by_name(std::string_view name) const {
        for (auto &n : namespaces)
            if (n.name == name) return &n;
        return nullptr;
    }
    uint64_t host_bytes() const {
        return vbytes(node_h) + vbytes(node_kh) + vbytes(node_flags) + vbytes(key_off) + vbytes(keys) + index.bytes() +
               vbytes(frow_node) + vbytes(frow_begin) + vbytes(fcol) + vbytes(rsub) + vbytes(rgrp) + vbytes(local) +
               vbytes(q_hash) + vbytes(lf_off) + vbytes(lr_off) + vbytes(lb_off) + vbytes(lf_col) + vbytes(lr_col) +
               vbytes(lb_col);
    }
    // register an owned node (registration index); a different key under the same hash is
    // a collision
    uint32_t reg(uint64_t h, const std::string &key, uint64_t kh, uint8_t flags) {
        bool fresh = false;
        const uint32_t idx = index.get_or_insert(h, (uint32_t)node_h.size(), fresh);
        if (fresh) {
            node_h.push_back(h);
            node_kh.push_back(kh);
            node_flags.push_back(flags);
            key_off.push_back(keys.size());
            keys.insert(keys.end(), key.begin(), key.end());
            return idx;
        }
        const uint64_t b = key_off[idx], e = idx + 1 < key_off.size() ? key_off[idx + 1] : keys.size();
        if (e - b != key.size() || memcmp(keys.data() + b, key.data(), key.size()))
            throw Error(KETOGPU_ECOLLISION, "64-bit node hash collision on rank " + std::to_string(rank) +
                                                ": reload with another ketogpu_shard_opts.salt");
        node_flags[idx] |= flags;
        return idx;
    }
};

struct ketogpu_shard_builder {
    std::unique_ptr<ketogpu_shard> s;
    std::chrono::steady_clock::time_point t0;
    bool has_empty_name_ns = false, odd_ns_names = false;
    // the open group
    bool open = false;
    int32_t g_ns = 0;
    std::string g_obj, g_rel;
    uint64_t g_h = 0;
    bool g_owned = false, g_known = false;
    int64_t first_bad = -1;
    uint64_t g_rows = 0;
    // its rows (valid prefix so far): subject hash, owned flag; owned subjects' keys
    std::vector<uint64_t> r_h, r_kh;
    std::vector<uint8_t> r_flags;  // kSet for subject-set subjects, 0x80 owned
    std::vector<uint64_t> r_key_off;
    std::string r_keys;
    std::string key, skey;
    uint64_t rows = 0, bad_rows = 0;

    bool ns_known(int32_t id) const { return s->ns_by_id(id) != nullptr; }

    // Subject.String() (definitions.go:164-170) key hash of a subject set / subject id
    uint64_t string_key_set(int32_t ns, std::string_view obj, std::string_view rel) {
        const Namespace *n = s->ns_by_id(ns);
        skey.assign(n ? n->name : std::string());
        skey.push_back(':');
        skey.append(obj.data(), obj.size());
        skey.push_back('#');
        skey.append(rel.data(), rel.size());
        return absorb(mix64(s->salt ^ 0x535452494e474b59ull), skey.data(), skey.size());
    }
    uint64_t string_key_id(std::string_view sid) {
        return absorb(mix64(s->salt ^ 0x535452494e474b59ull), sid.data(), sid.size());
    }

    void wildcard(const char *what) {
        throw Error(KETOGPU_EINVAL, std::string("partitioned loader: ") + what +
                                        " is a wildcard subject set (R5: its rows are the union of many groups); "
                                        "load this network with the whole-graph snapshot");
    }

    void close_group() {
        if (!open) return;
        open = false;
        ketogpu_shard &S = *s;
        if (!g_known) return;  // a group of an unknown namespace is no node (all its rows are bad)
        // R7: the check engine sees the rows before the poisoned page
        const uint64_t ps = (uint64_t)S.page_size;
        const uint64_t len = first_bad < 0 ? r_h.size() : std::min<uint64_t>(r_h.size(), (uint64_t)first_bad / ps * ps);
        uint32_t gi = NONE;
        if (g_owned) {
            key_set(key, g_ns, g_obj, g_rel);
            gi = S.reg(g_h, key, string_key_set(g_ns, g_obj, g_rel), (uint8_t)(kSet | (len ? kExp : 0)));
            // the same group closed before (the key matched: not a hash collision)
            if (S.node_flags[gi] & kClosed)
                throw Error(KETOGPU_EINVAL, "rows are not in ORDER BY order: a group (namespace_id, object, relation) "
                                            "appears twice in the stream");
            S.node_flags[gi] |= kClosed;
            if (len) {
                S.frow_node.push_back(gi);
                S.frow_begin.push_back(S.fcol.size());
                S.fcol.insert(S.fcol.end(), r_h.begin(), r_h.begin() + len);
            }
        }
        for (uint64_t i = 0; i < len; i++) {
            if (!(r_flags[i] & 0x80)) continue;
            const uint64_t b = r_key_off[i], e = r_key_off[i + 1];
            key.assign(r_keys.data() + b, e - b);
            const uint32_t si = S.reg(r_h[i], key, r_kh[i], (uint8_t)((r_flags[i] & kSet) | kSub));
            S.rsub.push_back(si);
            S.rgrp.push_back(g_h);
        }
        S.stats.forward_edges += g_owned ? len : 0;
    }

    void open_group(int32_t ns, std::string_view obj, std::string_view rel) {
        open = true;
        g_ns = ns;
        g_obj.assign(obj.data(), obj.size());
        g_rel.assign(rel.data(), rel.size());
        key_set(key, ns, obj, rel);
        g_h = key_hash(s->salt, key);
        g_owned = s->owner_of_hash(g_h) == s->rank;
        g_known = ns_known(ns);
        if (g_known) {
            const Namespace *n = s->ns_by_id(ns);
            if (obj.empty() || rel.empty() || n->name.empty()) wildcard("a group with an empty field");
        }
        first_bad = -1;
        g_rows = 0;
        r_h.clear();
        r_kh.clear();
        r_flags.clear();
        r_key_off.assign(1, 0);
        r_keys.clear();
    }

    void add(const ketogpu_row_batch *r, size_t i, std::string_view obj, std::string_view rel) {
        const int32_t ns = r->namespace_id[i];
        if (!open || ns != g_ns || obj != g_obj || rel != g_rel) {
            close_group();
            open_group(ns, obj, rel);
        }
        rows++;
        const uint8_t kind = r->subject_kind[i] ? 1 : 0;
        int32_t ssns = 0;
        if (kind) {
            if (!r->ss_namespace_id || !r->ss_object_off || !r->ss_relation_off)
                throw Error(KETOGPU_EINVAL, "subject-set row without subject_set columns");
            ssns = r->ss_namespace_id[i];
        } else if (!r->subject_id_off) {
            throw Error(KETOGPU_EINVAL, "subject-id row without subject_id column");
        }
        // toInternal fails for unknown namespace ids (relationtuples.go:48-51,64-67)
        const bool bad = !g_known || (kind && !ns_known(ssns));
        if (bad) bad_rows++;
        if (first_bad < 0 && bad) first_bad = (int64_t)g_rows;
        g_rows++;
        if (first_bad >= 0) return;  // past the poisoned page's start: nothing is kept
        uint64_t h, kh;
        uint8_t fl;
        if (kind) {
            const std::string_view so = col(r->ss_object_data, r->ss_object_off, i);
            const std::string_view sr = col(r->ss_relation_data, r->ss_relation_off, i);
            if (so.empty() || sr.empty() || s->ns_by_id(ssns)->name.empty()) wildcard("a subject set with an empty field");
            key_set(key, ssns, so, sr);
            h = key_hash(s->salt, key);
            kh = string_key_set(ssns, so, sr);
            fl = kSet;
        } else {
            const std::string_view sid = col(r->subject_id_data, r->subject_id_off, i);
            key_id(key, sid);
            h = key_hash(s->salt, key);
            // only ids with both ':' and '#' can share a key with a subject set (R4)
            kh = sid.find(':') != std::string_view::npos && sid.find('#') != std::string_view::npos
                     ? string_key_id(sid)
                     : 0;
            fl = 0;
        }
        const bool owned = s->owner_of_hash(h) == s->rank;
        r_h.push_back(h);
        r_kh.push_back(kh);
        r_flags.push_back((uint8_t)(fl | (owned ? 0x80 : 0)));
        if (owned) r_keys.append(key);
        r_key_off.push_back(r_keys.size());
    }
};

namespace {

int fail(const Error &e) {
    set_last_error(e.what());
    return e.code;
}

#define SHARD_TRY try {
#define SHARD_END                                                                                      \
    }                                                                                                  \
    catch (const Error &e) {                                                                           \
        return fail(e);                                                                                \
    }                                                                                                  \
    catch (const std::bad_alloc &) {                                                                   \
        set_last_error("out of host memory");                                                          \
        return KETOGPU_ENOMEM;                                                                         \
    }                                                                                                  \
    return KETOGPU_OK;

// local numbering: interior, other expandable, the rest (registration order inside)
void number(ketogpu_shard &S) {
    const size_t n = S.node_h.size();
    S.local.assign(n, NONE);
    uint64_t c[3] = {0, 0, 0};
    auto cls = [&](size_t i) {
        const uint8_t f = S.node_flags[i];
        return (f & kExp) ? ((f & kSub) ? 0 : 1) : 2;
    };
    for (size_t i = 0; i < n; i++) c[cls(i)]++;
    uint64_t base[3] = {0, c[0], c[0] + c[1]};
    for (size_t i = 0; i < n; i++) S.local[i] = (uint32_t)base[cls(i)]++;
    S.nil = c[0];
    S.nxl = c[0] + c[1];
    S.nl = n;
}

}  // namespace

extern "C" {

int ketogpu_shard_builder_new(const ketogpu_namespace *namespaces, size_t num_namespaces,
                              const ketogpu_shard_opts *o, ketogpu_shard_builder **out) {
    SHARD_TRY
    if (!o || !out || (num_namespaces && !namespaces)) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    if (o->world < 1 || o->rank < 0 || o->rank >= o->world || o->world > 64)
        throw Error(KETOGPU_EINVAL, "shard: need 0 <= rank < world <= 64");
    if (o->page_size < 0) throw Error(KETOGPU_EINVAL, "negative page size");
    if (o->flags & ~(uint32_t)KETOGPU_ORDER_NULLS_LAST)
        throw Error(KETOGPU_EINVAL, "shard: rows must arrive in ORDER BY order (no KETOGPU_BUILD_SORT)");
    auto b = std::make_unique<ketogpu_shard_builder>();
    b->t0 = std::chrono::steady_clock::now();
    b->s = std::make_unique<ketogpu_shard>();
    ketogpu_shard &S = *b->s;
    for (size_t i = 0; i < num_namespaces; i++) {
        Namespace n{namespaces[i].id, namespaces[i].name ? namespaces[i].name : ""};
        for (auto &m : S.namespaces)  // first-match resolution needs unique names and ids (R11)
            if (m.id == n.id || m.name == n.name)
                throw Error(KETOGPU_EINVAL, "duplicate namespace name or id in configuration: " + n.name);
        S.namespaces.push_back(n);
    }
    S.page_size = o->page_size ? o->page_size : 100;
    S.rank = (uint32_t)o->rank;
    S.world = (uint32_t)o->world;
    S.salt = o->salt;
    *out = b.release();
    SHARD_END
}

void ketogpu_shard_builder_free(ketogpu_shard_builder *b) { delete b; }

int ketogpu_shard_builder_append(ketogpu_shard_builder *b, const ketogpu_row_batch *r) {
    SHARD_TRY
    if (!b || !r) throw Error(KETOGPU_EINVAL, "null argument");
    if (!r->n) return KETOGPU_OK;
    if (!r->namespace_id || !r->object_off || !r->relation_off || !r->subject_kind)
        throw Error(KETOGPU_EINVAL, "row batch misses a required column");
    for (size_t i = 0; i < r->n; i++)
        b->add(r, i, col(r->object_data, r->object_off, i), col(r->relation_data, r->relation_off, i));
    SHARD_END
}

int ketogpu_shard_builder_finish(ketogpu_shard_builder *b, ketogpu_shard **out) {
    std::unique_ptr<ketogpu_shard_builder> owned(b);
    SHARD_TRY
    if (!b || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    b->close_group();
    ketogpu_shard &S = *b->s;
    number(S);
    S.stats.rows = b->rows;
    S.stats.bad_rows = b->bad_rows;
    S.stats.owned_nodes = S.nl;
    S.stats.owned_interior = S.nil;
    S.stats.owned_expandable = S.nxl;
    S.stats.reverse_edges = S.rsub.size();
    S.stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - b->t0).count();
    S.stats.host_bytes = S.host_bytes();
    *out = b->s.release();
    SHARD_END
}

void ketogpu_shard_free(ketogpu_shard *s) { delete s; }

int ketogpu_shard_counts(const ketogpu_shard *s, uint64_t counts[3]) {
    SHARD_TRY
    if (!s || !counts) throw Error(KETOGPU_EINVAL, "null argument");
    counts[0] = s->nil;
    counts[1] = s->nxl - s->nil;
    counts[2] = s->nl - s->nxl;
    SHARD_END
}

int ketogpu_shard_set_layout(ketogpu_shard *s, const uint64_t *all) {
    SHARD_TRY
    if (!s || !all) throw Error(KETOGPU_EINVAL, "null argument");
    uint64_t m[3] = {0, 0, 0};
    for (uint32_t r = 0; r < s->world; r++)
        for (int c = 0; c < 3; c++) m[c] = std::max(m[c], all[3 * r + c]);
    if (all[3 * s->rank] != s->nil || all[3 * s->rank + 1] != s->nxl - s->nil || all[3 * s->rank + 2] != s->nl - s->nxl)
        throw Error(KETOGPU_EINVAL, "shard: the gathered counts do not hold this rank's own");
    const uint64_t W = s->world;
    s->Ni = W * m[0];
    s->Nx = s->Ni + W * m[1];
    s->N = s->Nx + W * m[2];
    if (s->N >= 0x80000000ull) throw Error(KETOGPU_EINVAL, "shard: more than 2^31 node ids (u32 device ids)");
    s->laid_out = true;
    // the id queries: every distinct hash this rank's rows reference, grouped by owner
    std::vector<uint64_t> q(s->fcol);
    q.insert(q.end(), s->rgrp.begin(), s->rgrp.end());
    std::sort(q.begin(), q.end());
    q.erase(std::unique(q.begin(), q.end()), q.end());
    s->q_count.assign(s->world, 0);
    for (uint64_t h : q) s->q_count[s->owner_of_hash(h)]++;
    std::vector<uint64_t> at(s->world, 0);
    for (uint32_t r = 1; r < s->world; r++) at[r] = at[r - 1] + s->q_count[r - 1];
    s->q_hash.assign(q.size(), 0);
    for (uint64_t h : q) s->q_hash[at[s->owner_of_hash(h)]++] = h;
    s->stats.queries = q.size();
    s->stats.host_bytes = std::max<uint64_t>(s->stats.host_bytes, s->host_bytes());
    SHARD_END
}

uint64_t ketogpu_shard_query_count(const ketogpu_shard *s) { return s ? s->q_hash.size() : 0; }

int ketogpu_shard_queries(const ketogpu_shard *s, uint64_t *hashes, uint64_t capacity, uint64_t *counts) {
    SHARD_TRY
    if (!s || !counts || (capacity && !hashes)) throw Error(KETOGPU_EINVAL, "null argument");
    if (!s->laid_out) throw Error(KETOGPU_EINVAL, "shard: ketogpu_shard_set_layout first");
    if (capacity < s->q_hash.size()) throw Error(KETOGPU_ENOMEM, "shard: query buffer too small");
    std::copy(s->q_hash.begin(), s->q_hash.end(), hashes);
    for (uint32_t r = 0; r < s->world; r++) counts[r] = s->q_count[r];
    SHARD_END
}

int ketogpu_shard_answer(const ketogpu_shard *s, const uint64_t *hashes, uint64_t n, uint32_t *ids) {
    SHARD_TRY
    if (!s || (n && (!hashes || !ids))) throw Error(KETOGPU_EINVAL, "null argument");
    if (!s->laid_out) throw Error(KETOGPU_EINVAL, "shard: ketogpu_shard_set_layout first");
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t idx = s->index.get(hashes[i]);
        if (idx == NONE || s->owner_of_hash(hashes[i]) != s->rank)
            throw Error(KETOGPU_EINVAL, "shard: asked for a node this rank does not own");
        ids[i] = (uint32_t)s->global_of_local(s->local[idx]);
    }
    SHARD_END
}

int ketogpu_shard_apply(ketogpu_shard *s, const uint32_t *ids, uint64_t n) {
    SHARD_TRY
    if (!s || (n && !ids)) throw Error(KETOGPU_EINVAL, "null argument");
    if (!s->laid_out || n != s->q_hash.size()) throw Error(KETOGPU_EINVAL, "shard: answers do not match the queries");
    ketogpu_shard &S = *s;
    HashIndex id_of;
    id_of.reserve(n);
    for (uint64_t i = 0; i < n; i++) {
        bool fresh;
        if (ids[i] >= S.N) throw Error(KETOGPU_EINVAL, "shard: an answered id is outside the layout");
        id_of.get_or_insert(S.q_hash[i], ids[i], fresh);
    }
    std::vector<uint64_t>().swap(S.q_hash);
    // forward rows over owned expandable locals [0, nxl): interior successors, sorted, unique
    S.lf_off.assign(S.nxl + 1, 0);
    std::vector<std::pair<uint32_t, uint64_t>> rows;  // (local, frow index)
    rows.reserve(S.frow_node.size());
    for (size_t k = 0; k < S.frow_node.size(); k++) rows.push_back({S.local[S.frow_node[k]], k});
    std::sort(rows.begin(), rows.end());
    std::vector<uint32_t> tmp;
    S.lf_col.clear();
    size_t k = 0;
    for (uint32_t l = 0; l < S.nxl; l++) {
        tmp.clear();
        for (; k < rows.size() && rows[k].first == l; k++) {
            const uint64_t f = rows[k].second;
            const uint64_t b = S.frow_begin[f], e = f + 1 < S.frow_begin.size() ? S.frow_begin[f + 1] : S.fcol.size();
            for (uint64_t j = b; j < e; j++) {
                const uint32_t v = id_of.get(S.fcol[j]);
                if (v < S.Ni) tmp.push_back(v);
            }
        }
        std::sort(tmp.begin(), tmp.end());
        tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
        S.lf_col.insert(S.lf_col.end(), tmp.begin(), tmp.end());
        S.lf_off[l + 1] = S.lf_col.size();
    }
    std::vector<uint64_t>().swap(S.fcol);
    std::vector<uint64_t>().swap(S.frow_begin);
    std::vector<uint32_t>().swap(S.frow_node);
    // reverse rows over every owned local [0, nl): expandable predecessors, sorted, unique
    // (interior predecessors first, as their ids are smaller)
    std::vector<std::pair<uint32_t, uint32_t>> rev(S.rsub.size());
    for (size_t i = 0; i < S.rsub.size(); i++) rev[i] = {S.local[S.rsub[i]], id_of.get(S.rgrp[i])};
    std::vector<uint32_t>().swap(S.rsub);
    std::vector<uint64_t>().swap(S.rgrp);
    id_of.clear();
    std::sort(rev.begin(), rev.end());
    rev.erase(std::unique(rev.begin(), rev.end()), rev.end());
    S.lr_off.assign(S.nl + 1, 0);
    S.lr_col.resize(rev.size());
    for (size_t i = 0; i < rev.size(); i++) {
        if (rev[i].second >= S.Nx) throw Error(KETOGPU_EINVAL, "shard: a group of a reverse row is not expandable");
        S.lr_off[rev[i].first + 1]++;
        S.lr_col[i] = rev[i].second;
    }
    for (uint64_t l = 0; l < S.nl; l++) S.lr_off[l + 1] += S.lr_off[l];
    // backward rows: the interior prefix of each owned interior node's reverse row
    S.lb_off.assign(S.nil + 1, 0);
    S.lb_col.clear();
    for (uint64_t l = 0; l < S.nil; l++) {
        const uint32_t *b = S.lr_col.data() + S.lr_off[l], *e = S.lr_col.data() + S.lr_off[l + 1];
        const uint32_t *m = std::lower_bound(b, e, (uint32_t)S.Ni);
        S.lb_col.insert(S.lb_col.end(), b, m);
        S.lb_off[l + 1] = S.lb_col.size();
    }
    S.stats.interior_forward_edges = S.lf_col.size();
    S.stats.reverse_edges = S.lr_col.size();
    S.ready = true;
    SHARD_END
}

uint64_t ketogpu_shard_claim_count(const ketogpu_shard *s) {
    if (!s) return 0;
    uint64_t n = 0;
    for (uint64_t kh : s->node_kh) n += kh != 0;
    return n;
}

int ketogpu_shard_claims(const ketogpu_shard *s, uint64_t *pairs, uint64_t capacity, uint64_t *counts) {
    SHARD_TRY
    if (!s || !counts || (capacity && !pairs)) throw Error(KETOGPU_EINVAL, "null argument");
    const uint64_t n = ketogpu_shard_claim_count(s);
    if (capacity < n) throw Error(KETOGPU_ENOMEM, "shard: claim buffer too small");
    std::vector<uint64_t> at(s->world, 0);
    for (uint32_t r = 0; r < s->world; r++) counts[r] = 0;
    for (uint64_t kh : s->node_kh)
        if (kh) counts[s->owner_of_hash(kh)]++;
    for (uint32_t r = 1; r < s->world; r++) at[r] = at[r - 1] + counts[r - 1];
    for (size_t i = 0; i < s->node_kh.size(); i++) {
        const uint64_t kh = s->node_kh[i];
        if (!kh) continue;
        uint64_t &p = at[s->owner_of_hash(kh)];
        pairs[2 * p] = kh;
        pairs[2 * p + 1] = s->node_h[i];
        p++;
    }
    SHARD_END
}

int ketogpu_shard_check_claims(ketogpu_shard *s, const uint64_t *pairs, uint64_t n, uint64_t *ambiguous) {
    SHARD_TRY
    if (!s || !ambiguous || (n && !pairs)) throw Error(KETOGPU_EINVAL, "null argument");
    std::vector<std::pair<uint64_t, uint64_t>> v(n);
    for (uint64_t i = 0; i < n; i++) v[i] = {pairs[2 * i], pairs[2 * i + 1]};
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    uint64_t amb = 0;
    for (size_t i = 1; i < v.size(); i++)
        if (v[i].first == v[i - 1].first) amb++;
    *ambiguous = amb;
    s->stats.ambiguous_keys = amb;
    std::vector<uint64_t>().swap(s->node_kh);
    SHARD_END
}

int ketogpu_shard_resolve_batch(const ketogpu_shard *s, const ketogpu_request_batch *q, uint32_t *roots,
                                uint32_t *targets, int32_t *status) {
    SHARD_TRY
    if (!s || !q || (q->n && (!roots || !targets))) throw Error(KETOGPU_EINVAL, "null argument");
    if (!s->ready) throw Error(KETOGPU_EINVAL, "shard: not loaded (ketogpu_shard_apply)");
    std::string key;
    for (size_t i = 0; i < q->n; i++) {
        if (status) status[i] = KETOGPU_OK;
        roots[i] = targets[i] = KETOGPU_NODE_NOT_OWNED;
        const uint8_t kind = q->subject_kind ? q->subject_kind[i] : 0;
        if (kind != 0 && kind != 1) {  // nil subject: ErrNilSubject
            roots[i] = targets[i] = NONE;
            if (status) status[i] = KETOGPU_EINVAL;
            continue;
        }
        const std::string_view ns = col(q->ns_data, q->ns_off, i), obj = col(q->obj_data, q->obj_off, i),
                               rel = col(q->rel_data, q->rel_off, i);
        if (ns.empty() || obj.empty() || rel.empty()) {  // wildcard root: not in the partitioned mode
            roots[i] = targets[i] = NONE;
            if (status) status[i] = KETOGPU_ENOTFOUND;
            continue;
        }
        const Namespace *n = s->ns_by_name(ns);
        if (!n) {  // unknown namespace: false (engine.go:75-77)
            roots[i] = targets[i] = NONE;
            continue;
        }
        key_set(key, n->id, obj, rel);
        uint64_t h = key_hash(s->salt, key);
        if (s->owner_of_hash(h) == s->rank) {
            const uint32_t idx = s->index.get(h);
            const uint64_t l = idx == NONE ? NONE : s->local[idx];
            roots[i] = l != NONE && l < s->nxl ? (uint32_t)s->global_of_local(l) : NONE;
        }
        if (kind == 0) {
            key_id(key, col(q->sid_data, q->sid_off, i));
        } else {
            const Namespace *sn = s->ns_by_name(col(q->ss_ns_data, q->ss_ns_off, i));
            if (!sn) {  // a subject set of an unknown namespace is in no row
                targets[i] = NONE;
                continue;
            }
            key_set(key, sn->id, col(q->ss_obj_data, q->ss_obj_off, i), col(q->ss_rel_data, q->ss_rel_off, i));
        }
        h = key_hash(s->salt, key);
        if (s->owner_of_hash(h) == s->rank) {
            const uint32_t idx = s->index.get(h);
            targets[i] = idx == NONE ? NONE : (uint32_t)s->global_of_local(s->local[idx]);
        }
    }
    SHARD_END
}

int ketogpu_shard_stats_get(const ketogpu_shard *s, ketogpu_shard_stats *out) {
    SHARD_TRY
    if (!s || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = s->stats;
    out->owned_nodes = s->nl;
    out->owned_interior = s->nil;
    out->owned_expandable = s->nxl;
    out->num_interior = s->Ni;
    out->num_expandable = s->Nx;
    out->num_nodes = s->N;
    SHARD_END
}

int ketogpu_shard_view(const ketogpu_shard *s, ketogpu_shard_graph *out) {
    SHARD_TRY
    if (!s || !out) throw Error(KETOGPU_EINVAL, "null argument");
    if (!s->ready) throw Error(KETOGPU_EINVAL, "shard: not loaded (ketogpu_shard_apply)");
    out->rank = s->rank;
    out->world = s->world;
    out->num_interior = (uint32_t)s->Ni;
    out->num_expandable = (uint32_t)s->Nx;
    out->num_nodes = (uint32_t)s->N;
    out->owned_interior = (uint32_t)s->nil;
    out->owned_expandable = (uint32_t)s->nxl;
    out->owned_nodes = (uint32_t)s->nl;
    out->lf_off = s->lf_off.data();
    out->lf_col = s->lf_col.data();
    out->lr_off = s->lr_off.data();
    out->lr_col = s->lr_col.data();
    out->lb_off = s->lb_off.data();
    out->lb_col = s->lb_col.data();
    SHARD_END
}

}  // extern "C"
