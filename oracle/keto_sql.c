/*
 * keto_sql — BASELINE / TEST INFRASTRUCTURE ONLY.
 *
 * The reference's check engine restated over a REAL SQLite database, issuing the
 * reference's own storage access for every subject-set expansion, on every CPU core the
 * caller gives it.  It shows the cost regime Keto runs in (one SQL round trip per page
 * per visited subject set), beside the in-memory oracle (keto_oracle.c) and the GPU.
 * Only bench.py's cpu_baseline leg and tests/ load it; the product never does.
 *
 * Restated (paths relative to the reference repository):
 *   GetRelationTuples   internal/persistence/sql/relationtuples.go:203-258: WHERE nid = ?
 *                       [AND relation = ?] [AND object = ?] [AND namespace_id = ?] (each
 *                       filter only when its field is non-empty, R5; the namespace name is
 *                       resolved last, an unknown one is herodot.ErrNotFound), ORDER BY of
 *                       :215, Paginate(page, 100) — pop's paginator counts the matching
 *                       rows (SELECT COUNT(*)) and reads LIMIT/OFFSET; the next page
 *                       exists while page < TotalPages (:243-246)
 *   toInternal          relationtuples.go:43-80 (namespace ids -> names; an unknown id
 *                       fails the whole page, R7)
 *   schema + indexes    migrations/templates/20210623162417_relationtuple.up.sql:3-48
 *   subjectIsAllowed    internal/check/engine.go:33-67, checkOneIndirectionFurther :69-91,
 *                       SubjectIsAllowed :93-95
 *   CheckAndAddVisited  internal/x/graph/graph_utils.go:13-35 (String() keys; a fresh map
 *                       per root tuple, ctx shadowed in the loop at engine.go:40)
 *
 * libsqlite3.so.0 is present on the host without its headers: the prototypes below are
 * the public sqlite3 C API's.  Every worker thread opens its own read-only connection to
 * the database file (readers run in parallel; the file lives in tmpfs).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct sqlite3 sqlite3;
typedef struct sqlite3_stmt sqlite3_stmt;
int sqlite3_open_v2(const char *filename, sqlite3 **db, int flags, const char *vfs);
int sqlite3_close(sqlite3 *db);
int sqlite3_exec(sqlite3 *db, const char *sql, int (*cb)(void *, int, char **, char **), void *arg, char **err);
int sqlite3_prepare_v2(sqlite3 *db, const char *sql, int n, sqlite3_stmt **stmt, const char **tail);
int sqlite3_bind_int(sqlite3_stmt *s, int i, int v);
int sqlite3_bind_int64(sqlite3_stmt *s, int i, long long v);
int sqlite3_bind_text(sqlite3_stmt *s, int i, const char *v, int n, void (*destructor)(void *));
int sqlite3_bind_null(sqlite3_stmt *s, int i);
int sqlite3_step(sqlite3_stmt *s);
int sqlite3_reset(sqlite3_stmt *s);
int sqlite3_finalize(sqlite3_stmt *s);
int sqlite3_column_type(sqlite3_stmt *s, int i);
int sqlite3_column_int(sqlite3_stmt *s, int i);
long long sqlite3_column_int64(sqlite3_stmt *s, int i);
const unsigned char *sqlite3_column_text(sqlite3_stmt *s, int i);
int sqlite3_column_bytes(sqlite3_stmt *s, int i);
const char *sqlite3_errmsg(sqlite3 *db);
int sqlite3_config(int op, ...);
#define SQLITE_CONFIG_MEMSTATUS 9
void sqlite3_free(void *p);
#define SQLITE_OK 0
#define SQLITE_ROW 100
#define SQLITE_DONE 101
#define SQLITE_NULL 5
#define SQLITE_OPEN_READONLY 0x1
#define SQLITE_OPEN_READWRITE 0x2
#define SQLITE_OPEN_CREATE 0x4
#define SQLITE_OPEN_NOMUTEX 0x8000
#define SQLITE_OPEN_URI 0x40
#define SQLITE_TRANSIENT ((void (*)(void *)) - 1)

#include "keto_sql.h"

#define NID "00000000-0000-0000-0000-00000000b2b2"
#define ORDER_BY                                                                                       \
    "nid, namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object, " \
    "subject_set_relation, commit_time"

typedef struct {
    int32_t id;
    char *name;
} ns_t;

struct ks_db {
    char *path;
    sqlite3 *w;  /* the loading connection */
    sqlite3_stmt *ins;
    ns_t *ns;
    size_t nns;
    int page_size;
    long long rows;
};

static const ns_t *ns_by_name(const ks_db *d, const char *name) {  /* namespace_memory.go:29-37 */
    for (size_t i = 0; i < d->nns; i++)
        if (!strcmp(d->ns[i].name, name)) return &d->ns[i];
    return NULL;
}
static const ns_t *ns_by_id(const ks_db *d, int32_t id) {  /* namespace_memory.go:39-47 */
    for (size_t i = 0; i < d->nns; i++)
        if (d->ns[i].id == id) return &d->ns[i];
    return NULL;
}

ks_db *ks_db_create(const char *path, int page_size) {
    /* no global allocation statistics: with them every malloc of every connection takes
     * one process-wide mutex and the worker threads serialize (must precede the first
     * connection; fails harmlessly once sqlite is initialized) */
    static int configured = 0;
    if (!configured) {
        configured = 1;
        sqlite3_config(SQLITE_CONFIG_MEMSTATUS, 0);
    }
    ks_db *d = calloc(1, sizeof *d);
    if (!d) return NULL;
    d->path = strdup(path);
    d->page_size = page_size > 0 ? page_size : 100;
    remove(path);
    if (sqlite3_open_v2(path, &d->w, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE, NULL) != SQLITE_OK) {
        ks_db_free(d);
        return NULL;
    }
    const char *schema =
        "PRAGMA journal_mode=OFF; PRAGMA synchronous=OFF;"
        "CREATE TABLE keto_relation_tuples (shard_id UUID NOT NULL, nid UUID NOT NULL, namespace_id INTEGER NOT NULL,"
        " object VARCHAR(64) NOT NULL, relation VARCHAR(64) NOT NULL, subject_id VARCHAR(64) NULL,"
        " subject_set_namespace_id INTEGER NULL, subject_set_object VARCHAR(64) NULL,"
        " subject_set_relation VARCHAR(64) NULL, commit_time TIMESTAMP NOT NULL, PRIMARY KEY (shard_id, nid),"
        " CONSTRAINT chk_keto_rt_subject_type CHECK ((subject_id IS NULL AND subject_set_namespace_id IS NOT NULL"
        " AND subject_set_object IS NOT NULL AND subject_set_relation IS NOT NULL) OR (subject_id IS NOT NULL AND"
        " subject_set_namespace_id IS NULL AND subject_set_object IS NULL AND subject_set_relation IS NULL)));"
        "BEGIN;";
    if (sqlite3_exec(d->w, schema, NULL, NULL, NULL) != SQLITE_OK ||
        sqlite3_prepare_v2(d->w,
                           "INSERT INTO keto_relation_tuples (shard_id, nid, namespace_id, object, relation, subject_id,"
                           " subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time)"
                           " VALUES (?, '" NID "', ?, ?, ?, ?, ?, ?, ?, ?)",
                           -1, &d->ins, NULL) != SQLITE_OK) {
        ks_db_free(d);
        return NULL;
    }
    return d;
}

int ks_db_add_namespace(ks_db *d, int32_t id, const char *name) {
    ns_t *n = realloc(d->ns, (d->nns + 1) * sizeof *n);
    if (!n) return KS_ENOMEM;
    d->ns = n;
    d->ns[d->nns].id = id;
    d->ns[d->nns].name = strdup(name);
    d->nns++;
    return KS_OK;
}

int ks_db_add_rows_columnar(ks_db *d, size_t n, const int32_t *ns, const char *obj, const uint64_t *obj_off,
                            const char *rel, const uint64_t *rel_off, const uint8_t *kind, const char *sid,
                            const uint64_t *sid_off, const int32_t *ss_ns, const char *ss_obj,
                            const uint64_t *ss_obj_off, const char *ss_rel, const uint64_t *ss_rel_off,
                            const int64_t *commit_time) {
    for (size_t i = 0; i < n; i++) {
        sqlite3_stmt *s = d->ins;
        char shard[32];
        snprintf(shard, sizeof shard, "%lld", d->rows++);
        sqlite3_bind_text(s, 1, shard, -1, SQLITE_TRANSIENT);
        sqlite3_bind_int(s, 2, ns[i]);
        sqlite3_bind_text(s, 3, obj + obj_off[i], (int)(obj_off[i + 1] - obj_off[i]), SQLITE_TRANSIENT);
        sqlite3_bind_text(s, 4, rel + rel_off[i], (int)(rel_off[i + 1] - rel_off[i]), SQLITE_TRANSIENT);
        if (kind[i] == 0) {
            sqlite3_bind_text(s, 5, sid + sid_off[i], (int)(sid_off[i + 1] - sid_off[i]), SQLITE_TRANSIENT);
            sqlite3_bind_null(s, 6);
            sqlite3_bind_null(s, 7);
            sqlite3_bind_null(s, 8);
        } else {
            sqlite3_bind_null(s, 5);
            sqlite3_bind_int(s, 6, ss_ns[i]);
            sqlite3_bind_text(s, 7, ss_obj + ss_obj_off[i], (int)(ss_obj_off[i + 1] - ss_obj_off[i]), SQLITE_TRANSIENT);
            sqlite3_bind_text(s, 8, ss_rel + ss_rel_off[i], (int)(ss_rel_off[i + 1] - ss_rel_off[i]), SQLITE_TRANSIENT);
        }
        sqlite3_bind_int64(s, 9, commit_time ? commit_time[i] : (long long)d->rows);
        const int rc = sqlite3_step(s);
        sqlite3_reset(s);
        if (rc != SQLITE_DONE) {
            fprintf(stderr, "keto_sql insert: %s\n", sqlite3_errmsg(d->w));
            return KS_EINVAL;
        }
    }
    return KS_OK;
}

int ks_db_finish(ks_db *d) {
    /* the reference's indexes (migrations/templates/20210623162417_relationtuple.up.sql:27-48) */
    const char *idx =
        "COMMIT;"
        "CREATE INDEX keto_relation_tuples_subject_ids_idx ON keto_relation_tuples (nid, namespace_id, object,"
        " relation, subject_id) WHERE subject_set_namespace_id IS NULL AND subject_set_object IS NULL AND"
        " subject_set_relation IS NULL;"
        "CREATE INDEX keto_relation_tuples_subject_sets_idx ON keto_relation_tuples (nid, namespace_id, object,"
        " relation, subject_set_namespace_id, subject_set_object, subject_set_relation) WHERE subject_id IS NULL;"
        "CREATE INDEX keto_relation_tuples_full_idx ON keto_relation_tuples (nid, namespace_id, object, relation,"
        " subject_id, subject_set_namespace_id, subject_set_object, subject_set_relation, commit_time);"
        "ANALYZE;";
    sqlite3_finalize(d->ins);
    d->ins = NULL;
    if (sqlite3_exec(d->w, idx, NULL, NULL, NULL) != SQLITE_OK) {
        fprintf(stderr, "keto_sql indexes: %s\n", sqlite3_errmsg(d->w));
        return KS_EINVAL;
    }
    sqlite3_close(d->w);
    d->w = NULL;
    return KS_OK;
}

void ks_db_free(ks_db *d) {
    if (!d) return;
    if (d->ins) sqlite3_finalize(d->ins);
    if (d->w) sqlite3_close(d->w);
    for (size_t i = 0; i < d->nns; i++) free(d->ns[i].name);
    free(d->ns);
    if (d->path) remove(d->path);
    free(d->path);
    free(d);
}

/* ------------------------------------------------------------------ a worker */
/* a set of String() keys (graph_utils.go:13-35) */
typedef struct {
    char **keys;
    uint64_t *hash;
    size_t cap, n;
} kset;

static uint64_t fnv(const char *s) {
    uint64_t h = 1469598103934665603ull;
    for (; *s; s++) h = (h ^ (unsigned char)*s) * 1099511628211ull;
    return h | 1;
}
static void kset_clear(kset *k) {
    for (size_t i = 0; i < k->cap; i++)
        if (k->keys[i]) free(k->keys[i]), k->keys[i] = NULL, k->hash[i] = 0;
    k->n = 0;
}
/* 1 if newly added, 0 if present */
static int kset_add(kset *k, const char *key) {
    if (2 * (k->n + 1) > k->cap) {
        kset o = *k;
        k->cap = o.cap ? 2 * o.cap : 64;
        k->keys = calloc(k->cap, sizeof *k->keys);
        k->hash = calloc(k->cap, sizeof *k->hash);
        k->n = 0;
        for (size_t i = 0; i < o.cap; i++)
            if (o.keys[i]) {
                size_t j = o.hash[i] & (k->cap - 1);
                while (k->keys[j]) j = (j + 1) & (k->cap - 1);
                k->keys[j] = o.keys[i];
                k->hash[j] = o.hash[i];
                k->n++;
            }
        free(o.keys);
        free(o.hash);
    }
    const uint64_t h = fnv(key);
    size_t j = h & (k->cap - 1);
    while (k->keys[j]) {
        if (k->hash[j] == h && !strcmp(k->keys[j], key)) return 0;
        j = (j + 1) & (k->cap - 1);
    }
    k->keys[j] = strdup(key);
    k->hash[j] = h;
    k->n++;
    return 1;
}

typedef struct { /* one row of a page, after toInternal */
    int is_set;
    char *a, *b, *c; /* subject id; or namespace name, object, relation */
} trow;

typedef struct {
    const ks_db *d;
    sqlite3 *c;
    sqlite3_stmt *count[8], *page[8]; /* by filter mask: bit 0 relation, 1 object, 2 namespace */
    kset *sets;
    size_t nsets;
    long long queries;
} worker;

static int prep(worker *w) {
    for (int m = 0; m < 8; m++) {
        char where[256] = "nid = '" NID "'";
        if (m & 1) strcat(where, " AND relation = ?");
        if (m & 2) strcat(where, " AND object = ?");
        if (m & 4) strcat(where, " AND namespace_id = ?");
        char q[1024];
        snprintf(q, sizeof q, "SELECT COUNT(*) FROM keto_relation_tuples WHERE %s", where);
        if (sqlite3_prepare_v2(w->c, q, -1, &w->count[m], NULL) != SQLITE_OK) return KS_EINVAL;
        snprintf(q, sizeof q,
                 "SELECT namespace_id, object, relation, subject_id, subject_set_namespace_id, subject_set_object,"
                 " subject_set_relation FROM keto_relation_tuples WHERE %s ORDER BY " ORDER_BY " LIMIT ? OFFSET ?",
                 where);
        if (sqlite3_prepare_v2(w->c, q, -1, &w->page[m], NULL) != SQLITE_OK) return KS_EINVAL;
    }
    return KS_OK;
}

static char *col(sqlite3_stmt *s, int i) {
    const unsigned char *t = sqlite3_column_text(s, i);
    return strdup(t ? (const char *)t : "");
}

/* GetRelationTuples(query, page): rows of the page, *has_next; KS_ENOTFOUND for an
 * unknown namespace name or a row with an unknown namespace id (the whole page errors) */
static int get_page(worker *w, const char *ns, const char *obj, const char *rel, int page, trow **out, int *nout,
                    int *has_next) {
    const int m = (rel[0] ? 1 : 0) | (obj[0] ? 2 : 0) | (ns[0] ? 4 : 0);
    int32_t nsid = 0;
    if (m & 4) {
        const ns_t *n = ns_by_name(w->d, ns);
        if (!n) return KS_ENOTFOUND;
        nsid = n->id;
    }
    sqlite3_stmt *st[2] = {w->count[m], w->page[m]};
    for (int k = 0; k < 2; k++) {
        int b = 1;
        if (m & 1) sqlite3_bind_text(st[k], b++, rel, -1, SQLITE_TRANSIENT);
        if (m & 2) sqlite3_bind_text(st[k], b++, obj, -1, SQLITE_TRANSIENT);
        if (m & 4) sqlite3_bind_int(st[k], b++, nsid);
        if (k == 1) {
            sqlite3_bind_int(st[k], b++, w->d->page_size);
            sqlite3_bind_int64(st[k], b++, (long long)(page - 1) * w->d->page_size);
        }
    }
    long long total = 0;
    if (sqlite3_step(st[0]) == SQLITE_ROW) total = sqlite3_column_int64(st[0], 0);
    sqlite3_reset(st[0]);
    const long long total_pages = (total + w->d->page_size - 1) / w->d->page_size;
    *has_next = page < total_pages;
    int cap = 16, n = 0, rc = KS_OK;
    trow *rows = malloc(cap * sizeof *rows);
    while (sqlite3_step(st[1]) == SQLITE_ROW) {
        if (!ns_by_id(w->d, sqlite3_column_int(st[1], 0))) rc = KS_ENOTFOUND; /* toInternal */
        if (n == cap) rows = realloc(rows, (cap *= 2) * sizeof *rows);
        trow *r = &rows[n++];
        memset(r, 0, sizeof *r);
        if (sqlite3_column_type(st[1], 3) != SQLITE_NULL) {
            r->a = col(st[1], 3);
        } else {
            const ns_t *sn = ns_by_id(w->d, sqlite3_column_int(st[1], 4));
            if (!sn) rc = KS_ENOTFOUND;
            r->is_set = 1;
            r->a = strdup(sn ? sn->name : "");
            r->b = col(st[1], 5);
            r->c = col(st[1], 6);
        }
    }
    sqlite3_reset(st[1]);
    w->queries += 2;
    *out = rows;
    *nout = n;
    return rc;
}

static void free_rows(trow *r, int n) {
    for (int i = 0; i < n; i++) free(r[i].a), free(r[i].b), free(r[i].c);
    free(r);
}

static void key_of(const trow *r, char *buf, size_t cap) { /* Subject.String(), definitions.go:164-170 */
    if (r->is_set)
        snprintf(buf, cap, "%s:%s#%s", r->a, r->b, r->c);
    else
        snprintf(buf, cap, "%s", r->a);
}

typedef struct {
    int is_set;
    const char *a, *b, *c;
} subj;

static int equals(const trow *r, const subj *s) { /* Subject.Equals, definitions.go:253-267 */
    if (r->is_set != s->is_set) return 0;
    if (!r->is_set) return !strcmp(r->a, s->a);
    return !strcmp(r->a, s->a) && !strcmp(r->b, s->b) && !strcmp(r->c, s->c);
}

static int one_further(worker *w, kset *visited, const subj *req, const char *ns, const char *obj, const char *rel,
                       int depth);

/* subjectIsAllowed (engine.go:33-67) over one page */
static int allowed_in(worker *w, kset *visited, const subj *req, const trow *rows, int n, int depth) {
    char key[1024];
    for (int i = 0; i < n; i++) {
        key_of(&rows[i], key, sizeof key);
        kset *child = visited;
        if (!visited) { /* no map in ctx: a fresh one for this root tuple (graph_utils.go:14-19) */
            if (depth >= (int)w->nsets) {
                w->sets = realloc(w->sets, (depth + 1) * sizeof *w->sets);
                memset(w->sets + w->nsets, 0, (depth + 1 - w->nsets) * sizeof *w->sets);
                w->nsets = depth + 1;
            }
            child = &w->sets[depth];
            kset_clear(child);
            kset_add(child, key);
        } else if (!kset_add(visited, key)) {
            continue;
        }
        if (equals(&rows[i], req)) return 1;
        if (!rows[i].is_set) continue;
        if (one_further(w, child, req, rows[i].a, rows[i].b, rows[i].c, depth + 1)) return 1;
    }
    return 0;
}

/* checkOneIndirectionFurther (engine.go:69-91) */
static int one_further(worker *w, kset *visited, const subj *req, const char *ns, const char *obj, const char *rel,
                       int depth) {
    for (int page = 1;; page++) {
        trow *rows = NULL;
        int n = 0, has_next = 0;
        const int rc = get_page(w, ns, obj, rel, page, &rows, &n, &has_next);
        if (rc) { /* ErrNotFound -> false (engine.go:75-77) */
            free_rows(rows, n);
            return 0;
        }
        const int a = allowed_in(w, visited, req, rows, n, depth);
        free_rows(rows, n);
        if (a || !has_next) return a;
    }
}

typedef struct {
    ks_db *d;
    size_t n;
    const char *const *ns, *const *obj, *const *rel, *const *sid, *const *ss_ns, *const *ss_obj, *const *ss_rel;
    const int *kind;
    uint8_t *allowed;
    int *status;
    double deadline;
    atomic_size_t next, done;
    atomic_llong queries;
} job;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *run(void *arg) {
    job *j = arg;
    worker w = {.d = j->d};
    /* immutable: the file does not change while checks run, so readers take no file locks */
    char uri[4200];
    snprintf(uri, sizeof uri, "file:%s?immutable=1", j->d->path);
    if (sqlite3_open_v2(uri, &w.c, SQLITE_OPEN_READONLY | SQLITE_OPEN_NOMUTEX | SQLITE_OPEN_URI, NULL) != SQLITE_OK ||
        /* the file is in tmpfs: map it instead of copying pages into a per-connection cache */
        sqlite3_exec(w.c, "PRAGMA mmap_size=17179869184; PRAGMA cache_size=-65536;", NULL, NULL, NULL) != SQLITE_OK ||
        prep(&w) != KS_OK) {
        fprintf(stderr, "keto_sql worker: %s\n", w.c ? sqlite3_errmsg(w.c) : "open failed");
        return NULL;
    }
    for (;;) {
        if (j->deadline > 0 && now_s() > j->deadline) break;
        const size_t i = atomic_fetch_add(&j->next, 1);
        if (i >= j->n) break;
        if (j->kind[i] < 0) {
            j->status[i] = KS_EINVAL;
            atomic_fetch_add(&j->done, 1);
            continue;
        }
        subj s = {j->kind[i], j->kind[i] ? j->ss_ns[i] : j->sid[i], j->ss_obj[i], j->ss_rel[i]};
        j->allowed[i] = (uint8_t)one_further(&w, NULL, &s, j->ns[i], j->obj[i], j->rel[i], 0);
        j->status[i] = KS_OK;
        atomic_fetch_add(&j->done, 1);
    }
    for (size_t k = 0; k < w.nsets; k++) {
        kset_clear(&w.sets[k]);
        free(w.sets[k].keys);
        free(w.sets[k].hash);
    }
    free(w.sets);
    for (int m = 0; m < 8; m++) sqlite3_finalize(w.count[m]), sqlite3_finalize(w.page[m]);
    sqlite3_close(w.c);
    atomic_fetch_add(&j->queries, w.queries);
    return NULL;
}

int ks_check_batch(ks_db *d, size_t n, const char *const *ns, const char *const *obj, const char *const *rel,
                   const int *kind, const char *const *sid, const char *const *ss_ns, const char *const *ss_obj,
                   const char *const *ss_rel, int nthreads, double seconds, uint8_t *allowed, int *status,
                   size_t *done, long long *queries) {
    job j = {.d = d, .n = n, .ns = ns, .obj = obj, .rel = rel, .sid = sid, .ss_ns = ss_ns, .ss_obj = ss_obj,
             .ss_rel = ss_rel, .kind = kind, .allowed = allowed, .status = status};
    atomic_init(&j.next, 0);
    atomic_init(&j.done, 0);
    atomic_init(&j.queries, 0);
    for (size_t i = 0; i < n; i++) status[i] = KS_SKIPPED;
    j.deadline = seconds > 0 ? now_s() + seconds : 0;
    if (nthreads < 1) nthreads = 1;
    pthread_t *t = calloc(nthreads, sizeof *t);
    for (int k = 0; k < nthreads; k++) pthread_create(&t[k], NULL, run, &j);
    for (int k = 0; k < nthreads; k++) pthread_join(t[k], NULL);
    free(t);
    if (done) *done = atomic_load(&j.done);
    if (queries) *queries = atomic_load(&j.queries);
    return KS_OK;
}
