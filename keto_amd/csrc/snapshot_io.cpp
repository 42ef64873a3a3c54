// snapshot_io.cpp — persisted snapshots: a versioned binary image
// of a finished Snapshot, so a restarted server maps its graph back in seconds instead
// of re-reading and re-interning every keto_relation_tuples row
// (internal/persistence/sql/relationtuples.go:203-258 read once per network).
//
// Layout: "KETOSNAP" | u32 format version | u32 sizeof(Group) | u32 sizeof(RowRef) |
// u32 sizeof(ketogpu_snapshot_stats) | then every field in a fixed order, vectors as
// u64 count + raw elements, string pools as u64 count + u32 lengths + bytes.  The
// derived hash maps (subject-set triples, subject-id index) are rebuilt on load.
#include <algorithm>
#include <cstdio>
#include <memory>

#include "ketogpu_internal.hpp"

using namespace ketogpu;

namespace {

constexpr char kMagic[8] = {'K', 'E', 'T', 'O', 'S', 'N', 'A', 'P'};
constexpr uint32_t kFormat = 4;  // 4: writable layout; 3: row order flag

struct File {
    FILE *f = nullptr;
    std::string path;
    uint64_t size = 0, pos = 0;  // read mode: file size and bytes consumed
    File(const char *p, const char *mode) : f(fopen(p, mode)), path(p) {
        if (!f) throw Error(KETOGPU_EINVAL, "cannot open " + path);
        if (mode[0] == 'r' && fseek(f, 0, SEEK_END) == 0) {
            const long n = ftell(f);
            size = n > 0 ? (uint64_t)n : 0;
            fseek(f, 0, SEEK_SET);
        }
    }
    ~File() {
        if (f) fclose(f);
    }
    void write(const void *p, size_t n) {
        if (n && fwrite(p, 1, n, f) != n) throw Error(KETOGPU_EINVAL, "short write to " + path);
    }
    void read(void *p, size_t n) {
        if (n && fread(p, 1, n, f) != n) throw Error(KETOGPU_EINVAL, "truncated snapshot file " + path);
        pos += n;
    }
    // a length field must fit in the rest of the file (a corrupt count must not allocate)
    void need(uint64_t count, uint64_t elem) {
        if (elem && count > (size - std::min(size, pos)) / elem)
            throw Error(KETOGPU_EINVAL, "corrupt length field in snapshot file " + path);
    }
    template <class T>
    void put(const T &v) {
        write(&v, sizeof v);
    }
    template <class T>
    T get() {
        T v;
        read(&v, sizeof v);
        return v;
    }
    template <class T>
    void put_vec(const std::vector<T> &v) {
        put<uint64_t>(v.size());
        write(v.data(), v.size() * sizeof(T));
    }
    template <class T>
    void get_vec(std::vector<T> &v) {
        uint64_t n = get<uint64_t>();
        need(n, sizeof(T));
        v.resize(n);
        read(v.data(), n * sizeof(T));
    }
    void put_str(std::string_view s) {
        put<uint32_t>((uint32_t)s.size());
        write(s.data(), s.size());
    }
    std::string get_str() {
        const uint32_t n = get<uint32_t>();
        need(n, 1);
        std::string s(n, '\0');
        read(s.data(), s.size());
        return s;
    }
    void put_pool(const StrPool &p) {
        put<uint64_t>(p.size());
        for (size_t i = 0; i < p.size(); i++) put_str(p.get((uint32_t)i));
    }
    void get_pool(StrPool &p) {
        uint64_t n = get<uint64_t>();
        need(n, sizeof(uint32_t));
        std::string s;
        for (uint64_t i = 0; i < n; i++) {
            s = get_str();
            if (p.intern(s.data(), s.size()) != (uint32_t)i)  // ids are intern order; id 0 is ""
                throw Error(KETOGPU_EINVAL, "corrupt string pool in " + path);
        }
    }
};

// Every index a loaded snapshot holds must stay inside the arrays it indexes: the host
// DFS, the resolver and the device kernels read them unchecked.  A file that passes the
// magic trailer but is corrupt (or written by a buggy writer) is refused here.
void validate(const Snapshot &s, const std::string &path) {
    auto bad = [&](const char *what) { throw Error(KETOGPU_EINVAL, path + ": inconsistent snapshot (" + what + ")"); };
    const uint64_t N = s.N, P = s.pool.size();
    if (!(s.Ni <= s.Nx && s.Nx <= s.N)) bad("node ranges");
    for (size_t n : {s.node_kind.size(), s.node_ns.size(), s.node_a.size(), s.node_b.size(), s.key_id.size(),
                     s.ambiguous.size(), s.node_row.size()})
        if (n != N) bad("per-node array size");
    for (uint64_t v = 0; v < N; v++) {
        if (s.node_kind[v] > 1 || s.node_a[v] >= P || (s.node_kind[v] == KETOGPU_SUBJECT_SET && s.node_b[v] >= P))
            bad("node identity");
        const RowRef &r = s.node_row[v];
        if (r.off > s.row_col.size() || r.len > s.row_col.size() - r.off || r.len > r.full_len) bad("node rows");
    }
    for (uint32_t x : s.sid_node)
        if (x != NONE && x >= N) bad("subject-id index");
    for (uint32_t x : s.row_col)
        if (x >= N) bad("row entries");
    for (uint32_t x : s.group_col)
        if (x >= N) bad("group entries");
    for (const Group &g : s.groups) {
        if (g.obj >= P || g.rel >= P || g.valid > g.full_len || g.begin > s.group_col.size() ||
            g.valid > s.group_col.size() - g.begin)
            bad("group rows");
        if (g.first_bad >= 0 && ((uint64_t)g.first_bad >= g.full_len || g.tail > s.tail_rows.size() ||
                                 g.full_len - (uint64_t)g.first_bad > s.tail_rows.size() - g.tail))
            bad("group tail");
    }
    for (const TupleRow &t : s.tail_rows)
        if (t.obj >= P || t.rel >= P || t.kind > 1 || (t.kind ? (t.ss_obj >= P || t.ss_rel >= P) : t.sid >= P))
            bad("tail rows");
    auto csr = [&](const std::vector<uint64_t> &off, const std::vector<uint32_t> &col, uint64_t rows, uint64_t lim,
                   const char *what) {
        if (off.size() != rows + 1 || off[0] != 0 || off.back() != col.size()) bad(what);
        for (uint64_t i = 0; i < rows; i++)
            if (off[i] > off[i + 1]) bad(what);
        for (uint32_t x : col)
            if (x >= lim) bad(what);
    };
    csr(s.fint_off, s.fint_col, s.Nx, s.Ni, "forward rows");
    if (s.writable) {
        if (!(s.n_cap >= N && s.Df < s.Ni && s.Dbi < s.Ni && s.Dbo >= s.Ni && s.Dbo < s.Nx)) bad("writable layout");
        csr(s.rev_off, s.rev_col, s.n_cap, s.Nx, "reverse rows");
    } else {
        csr(s.rev_off, s.rev_col, N, s.Nx, "reverse rows");
    }
    if (s.has_ambiguous && s.row_amb.size() < ((uint64_t)s.Nx + 31) / 32) bad("ambiguous-row bitmap");
}

}  // namespace

extern "C" {

int ketogpu_snapshot_save(const ketogpu_snapshot *sp, const char *path) {
    try {
        if (!sp || !path) throw Error(KETOGPU_EINVAL, "null argument");
        const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
        std::shared_lock<std::shared_mutex> rd(s.mu);
        File f(path, "wb");
        f.write(kMagic, sizeof kMagic);
        f.put<uint32_t>(kFormat);
        f.put<uint32_t>(sizeof(Group));
        f.put<uint32_t>(sizeof(RowRef));
        f.put<uint32_t>(sizeof(ketogpu_snapshot_stats));
        f.put<uint64_t>(s.namespaces.size());
        for (const Namespace &n : s.namespaces) {
            f.put<int32_t>(n.id);
            f.put_str(n.name);
        }
        f.put<int32_t>(s.page_size);
        f.put<uint8_t>(s.nulls_last);
        f.put<int32_t>(s.empty_name_ns);
        f.put<uint8_t>(s.has_empty_name_ns);
        f.put_pool(s.pool);
        f.put_vec(s.groups);
        f.put_vec(s.group_col);
        f.put_vec(s.tail_rows);
        f.put<uint32_t>(s.N);
        f.put<uint32_t>(s.Ni);
        f.put<uint32_t>(s.Nx);
        f.put_vec(s.node_kind);
        f.put_vec(s.node_ns);
        f.put_vec(s.node_a);
        f.put_vec(s.node_b);
        f.put_vec(s.sid_node);
        f.put_vec(s.node_row);
        f.put_vec(s.row_col);
        f.put_vec(s.key_id);
        f.put_vec(s.ambiguous);
        f.put_pool(s.key_pool);
        f.put<uint8_t>(s.has_ambiguous);
        f.put_vec(s.fint_off);
        f.put_vec(s.fint_col);
        f.put_vec(s.rev_off);
        f.put_vec(s.rev_col);
        f.put_vec(s.row_amb);
        f.put<uint8_t>(s.writable);
        f.put<uint32_t>(s.Df);
        f.put<uint32_t>(s.Dbi);
        f.put<uint32_t>(s.Dbo);
        f.put<uint32_t>(s.n_cap);
        f.put<uint64_t>(s.row_garbage);
        f.put(s.stats);
        f.write(kMagic, sizeof kMagic);  // trailer: a complete file ends with the magic again
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

int ketogpu_snapshot_load(const char *path, ketogpu_snapshot **out) {
    try {
        if (!path || !out) throw Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        File f(path, "rb");
        char magic[8];
        f.read(magic, sizeof magic);
        if (memcmp(magic, kMagic, sizeof magic)) throw Error(KETOGPU_EINVAL, std::string(path) + " is not a snapshot");
        if (f.get<uint32_t>() != kFormat || f.get<uint32_t>() != sizeof(Group) || f.get<uint32_t>() != sizeof(RowRef) ||
            f.get<uint32_t>() != sizeof(ketogpu_snapshot_stats))
            throw Error(KETOGPU_EINVAL, std::string(path) + ": snapshot format of another library version");
        auto s = std::make_unique<Snapshot>();
        uint64_t nns = f.get<uint64_t>();
        for (uint64_t i = 0; i < nns; i++) {
            Namespace n;
            n.id = f.get<int32_t>();
            n.name = f.get_str();
            s->namespaces.push_back(std::move(n));
        }
        s->page_size = f.get<int32_t>();
        s->nulls_last = f.get<uint8_t>() != 0;
        s->empty_name_ns = f.get<int32_t>();
        s->has_empty_name_ns = f.get<uint8_t>() != 0;
        s->pool = StrPool();
        f.get_pool(s->pool);
        f.get_vec(s->groups);
        f.get_vec(s->group_col);
        f.get_vec(s->tail_rows);
        s->N = f.get<uint32_t>();
        s->Ni = f.get<uint32_t>();
        s->Nx = f.get<uint32_t>();
        f.get_vec(s->node_kind);
        f.get_vec(s->node_ns);
        f.get_vec(s->node_a);
        f.get_vec(s->node_b);
        f.get_vec(s->sid_node);
        f.get_vec(s->node_row);
        f.get_vec(s->row_col);
        f.get_vec(s->key_id);
        f.get_vec(s->ambiguous);
        s->key_pool = StrPool();
        f.get_pool(s->key_pool);
        s->has_ambiguous = f.get<uint8_t>() != 0;
        f.get_vec(s->fint_off);
        f.get_vec(s->fint_col);
        f.get_vec(s->rev_off);
        f.get_vec(s->rev_col);
        f.get_vec(s->row_amb);
        s->writable = f.get<uint8_t>() != 0;
        s->Df = f.get<uint32_t>();
        s->Dbi = f.get<uint32_t>();
        s->Dbo = f.get<uint32_t>();
        s->n_cap = f.get<uint32_t>();
        s->row_garbage = f.get<uint64_t>();
        s->stats = f.get<ketogpu_snapshot_stats>();
        f.read(magic, sizeof magic);
        if (memcmp(magic, kMagic, sizeof magic)) throw Error(KETOGPU_EINVAL, std::string(path) + ": truncated snapshot");
        validate(*s, path);
        for (uint32_t v = 0; v < s->N; v++)  // the subject-set index (sid_node is stored)
            if (s->node_kind[v] == KETOGPU_SUBJECT_SET) s->set_node.get_or_insert(s->node_ns[v], s->node_a[v], s->node_b[v], v);
        if (s->writable) index_groups(*s);
        *out = reinterpret_cast<ketogpu_snapshot *>(s.release());
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

}  // extern "C"
