// snapshot_io.cpp — persisted snapshots: a versioned binary image
// of a finished Snapshot, so a restarted server maps its graph back in seconds instead
// of re-reading and re-interning every keto_relation_tuples row
// (internal/persistence/sql/relationtuples.go:203-258 read once per network).
//
// Layout: "KETOSNAP" | u32 format version | u32 sizeof(Group) | u32 sizeof(RowRef) |
// u32 sizeof(ketogpu_snapshot_stats) | then every field in a fixed order, vectors as
// u64 count + raw elements, string pools as u64 count + u32 lengths + bytes.  The
// derived hash maps (subject-set triples, subject-id index) are rebuilt on load.
#include <cstdio>
#include <memory>

#include "ketogpu_internal.hpp"

using namespace ketogpu;

namespace {

constexpr char kMagic[8] = {'K', 'E', 'T', 'O', 'S', 'N', 'A', 'P'};
constexpr uint32_t kFormat = 3;  // 3: row order flag

struct File {
    FILE *f = nullptr;
    std::string path;
    File(const char *p, const char *mode) : f(fopen(p, mode)), path(p) {
        if (!f) throw Error(KETOGPU_EINVAL, "cannot open " + path);
    }
    ~File() {
        if (f) fclose(f);
    }
    void write(const void *p, size_t n) {
        if (n && fwrite(p, 1, n, f) != n) throw Error(KETOGPU_EINVAL, "short write to " + path);
    }
    void read(void *p, size_t n) {
        if (n && fread(p, 1, n, f) != n) throw Error(KETOGPU_EINVAL, "truncated snapshot file " + path);
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
        v.resize(n);
        read(v.data(), n * sizeof(T));
    }
    void put_str(std::string_view s) {
        put<uint32_t>((uint32_t)s.size());
        write(s.data(), s.size());
    }
    std::string get_str() {
        std::string s(get<uint32_t>(), '\0');
        read(s.data(), s.size());
        return s;
    }
    void put_pool(const StrPool &p) {
        put<uint64_t>(p.size());
        for (size_t i = 0; i < p.size(); i++) put_str(p.get((uint32_t)i));
    }
    void get_pool(StrPool &p) {
        uint64_t n = get<uint64_t>();
        std::string s;
        for (uint64_t i = 0; i < n; i++) {
            s = get_str();
            if (p.intern(s.data(), s.size()) != (uint32_t)i)  // ids are intern order; id 0 is ""
                throw Error(KETOGPU_EINVAL, "corrupt string pool in " + path);
        }
    }
};

}  // namespace

extern "C" {

int ketogpu_snapshot_save(const ketogpu_snapshot *sp, const char *path) {
    try {
        if (!sp || !path) throw Error(KETOGPU_EINVAL, "null argument");
        const Snapshot &s = *reinterpret_cast<const Snapshot *>(sp);
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
        s->stats = f.get<ketogpu_snapshot_stats>();
        f.read(magic, sizeof magic);
        if (memcmp(magic, kMagic, sizeof magic)) throw Error(KETOGPU_EINVAL, std::string(path) + ": truncated snapshot");
        if (s->node_kind.size() != s->N || s->fint_off.size() != (size_t)s->Nx + 1 || s->rev_off.size() != (size_t)s->N + 1)
            throw Error(KETOGPU_EINVAL, std::string(path) + ": inconsistent snapshot");
        for (uint32_t v = 0; v < s->N; v++)  // the subject-set index (sid_node is stored)
            if (s->node_kind[v] == KETOGPU_SUBJECT_SET) s->set_node.get_or_insert(s->node_ns[v], s->node_a[v], s->node_b[v], v);
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
