// ketogpu_internal.hpp — shared host-side data structures of libketogpu.
//
// The snapshot is the device-ready restatement of the reference's tuple table:
//   * rows are grouped per (namespace_id, object, relation) in the backend's ORDER BY
//     order (internal/persistence/sql/relationtuples.go:215),
//   * every subject becomes an interned node (SubjectID or SubjectSet,
//     internal/relationtuple/definitions.go:39-41,103-118),
//   * a subject set expands into the rows its query returns, with empty fields acting
//     as "no filter" (relationtuples.go:218-236) and page-poison truncation for rows
//     whose namespace ids are not configured (relationtuples.go:43-80,248-255),
//   * node ids are ordered interior | source | non-expandable so the device traversal
//     state only covers interior nodes (DESIGN.md "Data layout in HBM").
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/ketogpu.h"

namespace ketogpu {

constexpr uint32_t NONE = KETOGPU_NODE_NONE;

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

inline uint64_t hash_bytes(const char *p, size_t n) {
    // 64-bit FNV-1a with a final avalanche; good enough for interning.
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    return h;
}

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

// Interned byte strings with stable storage.  id 0 is always "".
class StrPool {
  public:
    StrPool() { intern("", 0); }
    uint32_t intern(const char *p, size_t n);
    uint32_t find(const char *p, size_t n) const;
    uint32_t find(std::string_view s) const { return find(s.data(), s.size()); }
    std::string_view get(uint32_t id) const { return std::string_view(ptr_[id], len_[id]); }
    size_t size() const { return ptr_.size(); }

  private:
    void rehash();
    std::vector<std::unique_ptr<char[]>> chunks_;
    size_t used_ = 0, cap_ = 0;
    std::vector<const char *> ptr_;
    std::vector<uint32_t> len_;
    std::vector<uint64_t> slot_hash_;
    std::vector<uint32_t> slot_id_;  // id+1, 0 = empty
    size_t mask_ = 0;
};

// Open-addressing map from a 96-bit key (int32 namespace id, u32 object id, u32 relation id)
// to a u32 value.
class TripleMap {
  public:
    TripleMap() { resize(1024); }
    uint32_t get(int32_t ns, uint32_t obj, uint32_t rel) const;
    // returns existing value or inserts `v` and returns it
    uint32_t get_or_insert(int32_t ns, uint32_t obj, uint32_t rel, uint32_t v);
    void remap(const std::vector<uint32_t> &perm);
    size_t size() const { return n_; }

  private:
    struct Slot {
        int32_t ns;
        uint32_t obj, rel, val;  // val == NONE: empty
    };
    static uint64_t h(int32_t ns, uint32_t obj, uint32_t rel) {
        return mix64(((uint64_t)(uint32_t)ns << 32 | obj) ^ mix64(rel + 0x9e3779b97f4a7c15ull));
    }
    void resize(size_t cap);
    std::vector<Slot> slots_;
    size_t n_ = 0, mask_ = 0;
};

struct Namespace {
    int32_t id;
    std::string name;
};

// One keto_relation_tuples row with interned strings (StrPool ids); kind 0 = subject id
// row (sid), 1 = subject-set row (ss_*).  seq orders equal keys (commit_time).
struct TupleRow {
    int32_t ns, ss_ns;
    uint32_t obj, rel, sid, ss_obj, ss_rel;
    uint8_t kind;
    uint64_t seq;
};

// One (namespace_id, object, relation) group of rows, in DB order.
struct Group {
    int32_t ns;
    uint32_t obj, rel;       // StrPool ids
    uint32_t cap;            // writable snapshots: slots reserved at begin / the row_col copy (0: valid)
    uint64_t begin;          // into Snapshot::group_col (valid prefix only)
    uint32_t valid;          // rows before the first bad row
    uint32_t full_len;       // all rows of the group
    int64_t first_bad;       // index of the first row with an unknown namespace, or -1
    uint64_t tail;           // into Snapshot::tail_rows: rows [first_bad, full_len) (kept for updates)
};

// Query result of one subject set / root query after page-poison truncation.
struct RowRef {
    uint64_t off = 0;        // into Snapshot::row_col
    uint32_t len = 0;        // rows returned to the check engine (truncated)
    uint32_t full_len = 0;   // rows of the query (for expand)
    int64_t first_bad = -1;  // index of first bad row in query order, -1 if none
};

struct ReachLabels;  // labels.hpp

struct Snapshot {
    // ---- configuration
    std::vector<Namespace> namespaces;  // config order, unique names and ids
    int page_size = 100;
    bool nulls_last = false;            // KETOGPU_ORDER_NULLS_LAST: the backend's row order
    int32_t empty_name_ns = 0;          // id of the namespace named "" (if has_empty_name_ns)
    bool has_empty_name_ns = false;

    // ---- strings and groups
    StrPool pool;
    std::vector<Group> groups;          // DB order
    std::vector<uint32_t> group_col;    // subjects (node ids) of the groups' valid prefixes
    std::vector<TupleRow> tail_rows;    // rows from each group's first bad row on

    // ---- nodes: [0, Ni) interior, [Ni, Nx) source-expandable, [Nx, N) non-expandable
    uint32_t N = 0, Ni = 0, Nx = 0;
    std::vector<uint8_t> node_kind;     // KETOGPU_SUBJECT_ID / _SET
    std::vector<int32_t> node_ns;       // set: namespace id
    std::vector<uint32_t> node_a;       // id: StrPool id of the subject id; set: object id
    std::vector<uint32_t> node_b;       // set: relation id
    std::vector<uint32_t> sid_node;     // StrPool id -> subject-id node (NONE)
    TripleMap set_node;                 // (ns, obj, rel) -> subject-set node
    std::vector<RowRef> node_row;       // per node: its query's rows (host DFS)
    std::vector<uint32_t> row_col;      // rows of wildcard queries (materialized) + copies
    std::vector<uint32_t> key_id;       // Subject.String() identity per node
    std::vector<uint8_t> ambiguous;     // key shared with another node (R4)
    StrPool key_pool;                   // keys that may collide (see snapshot.cpp)
    bool has_ambiguous = false;

    // ---- device graph (built on host, uploaded by the engine)
    std::vector<uint64_t> fint_off;     // Nx + 1
    std::vector<uint32_t> fint_col;     // interior successors, sorted, unique
    std::vector<uint64_t> rev_off;      // N + 1
    std::vector<uint32_t> rev_col;      // expandable predecessors, sorted, unique
    std::vector<uint32_t> row_amb;      // bitmap over Nx: row contains an ambiguous node

    ketogpu_snapshot_stats stats{};

    // ---- writable layout (KETOGPU_BUILD_WRITABLE, snapshot_write.cpp)
    // Device rows carry free slots filled with placeholder nodes that have no rows and no
    // names: Df (interior, the largest interior id) pads forward rows, Dbi (interior, the
    // next smaller id) pads the interior part of reverse rows and Dbo (the largest
    // expandable id) their other part.  The forward search can only reach Df and the
    // backward search only Dbi/Dbo, so a meet or a pull never happens at a placeholder and
    // sorted rows stay sorted.  Ids [N, n_cap) are reserved for new subjects (reverse rows
    // of only free slots).
    bool writable = false;
    uint32_t Df = NONE, Dbi = NONE, Dbo = NONE, n_cap = 0;
    TripleMap group_idx;                // (namespace id, object, relation) -> index into groups
    uint64_t version = 0;               // writes applied in place
    uint64_t row_garbage = 0;           // stale group rows left by grown groups (group_col, row_col)
    struct Patch {
        uint8_t rev;                    // 0: forward row of node, 1: reverse row
        uint32_t node;
    };
    std::vector<Patch> patches;         // device rows changed, in write order (engines replay)
    uint64_t patch_base = 0;            // patches trimmed off the front (absolute index of patches[0])
    // engines over this snapshot -> the absolute patch position each has replayed up to;
    // a write trims the log below the smallest
    mutable std::mutex readers_mu;
    mutable std::map<const void *, uint64_t> readers;
    void reader_at(const void *who, uint64_t pos) const {
        std::lock_guard<std::mutex> lk(readers_mu);
        readers[who] = pos;
    }
    void reader_gone(const void *who) const {
        std::lock_guard<std::mutex> lk(readers_mu);
        readers.erase(who);
    }
    uint64_t patch_end() const { return patch_base + patches.size(); }
    // under the exclusive write lock: drop what every engine has replayed
    void trim_patches() {
        uint64_t lo = patch_end();
        {
            std::lock_guard<std::mutex> lk(readers_mu);
            for (auto &kv : readers) lo = std::min(lo, kv.second);
        }
        if (lo > patch_base) {
            patches.erase(patches.begin(), patches.begin() + (ptrdiff_t)(lo - patch_base));
            patch_base = lo;
        }
    }
    mutable std::shared_mutex mu;       // writes exclusive; engine, resolve and expand calls shared
    // derived indexes built once per snapshot VERSION and shared by its engines (labels.cpp
    // reach_labels_of: a writable snapshot's writes bump the version, so a later engine sync
    // or relabel rebuilds them).  derived_mu guards only the cache and the in-flight build's
    // future: the build itself runs outside it, and engines asking for the same version while
    // it runs wait on that future instead of building again
    mutable std::mutex derived_mu;
    mutable std::shared_ptr<const ReachLabels> reach_cache;
    mutable std::shared_future<std::shared_ptr<const ReachLabels>> reach_building;
    mutable uint64_t reach_building_version = ~0ull;
    // An engine's way back to its snapshot at teardown: the snapshot's destructor clears it,
    // so an engine freed after its snapshot (a garbage collector's order) skips the
    // deregistration instead of touching freed memory.
    struct ReaderLink {
        std::mutex mu;
        const Snapshot *snap = nullptr;
    };
    std::shared_ptr<ReaderLink> link = std::make_shared<ReaderLink>();
    Snapshot() = default;
    Snapshot(const Snapshot &) = delete;
    Snapshot &operator=(const Snapshot &) = delete;
    ~Snapshot() {
        std::lock_guard<std::mutex> lk(link->mu);
        link->snap = nullptr;
    }

    // ---- helpers
    const Namespace *ns_by_name(std::string_view name) const {
        for (auto &n : namespaces)
            if (n.name == name) return &n;
        return nullptr;
    }
    const Namespace *ns_by_id(int32_t id) const {
        for (auto &n : namespaces)
            if (n.id == id) return &n;
        return nullptr;
    }
    const uint32_t *row_ptr(uint32_t v) const { return row_col.data() + node_row[v].off; }
    std::string key_string(uint32_t v) const;
    // Materialize the rows of a query with "" = no filter.  ns_filter < 0 = any.
    RowRef materialize(bool any_ns, int32_t ns, uint32_t obj, bool any_obj, uint32_t rel,
                       bool any_rel, std::vector<uint32_t> &out) const;
};

// writable layout: pad the compact device rows (snapshot_write.cpp)
void make_writable(Snapshot &s);
void index_groups(Snapshot &s);  // group_idx from groups

// ---- host engine entry points (host_engine.cpp)
struct ResolvedRoot {
    enum Kind { EMPTY, NODE, DYNAMIC, UNKNOWN_NS } kind = EMPTY;
    uint32_t node = NONE;
    // DYNAMIC: the query, to materialize
    bool any_ns = false, any_obj = false, any_rel = false;
    int32_t ns = 0;
    uint32_t obj = 0, rel = 0;
};
ResolvedRoot resolve_root(const Snapshot &s, std::string_view ns, std::string_view obj, std::string_view rel);
uint32_t resolve_subject(const Snapshot &s, int kind, std::string_view id, std::string_view ns, std::string_view obj,
                         std::string_view rel);
uint32_t resolve_subject(const Snapshot &s, const ketogpu_subject &subj);
inline std::string_view sv(const char *p) { return p ? std::string_view(p) : std::string_view(); }
// exact sequential check (reference DFS with Subject.String() visited keys)
bool exact_check(const Snapshot &s, const uint32_t *root_rows, uint32_t root_len,
                 const ketogpu_subject &req, uint32_t target);

}  // namespace ketogpu
