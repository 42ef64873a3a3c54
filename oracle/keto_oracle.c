/*
 * keto_oracle.c — TEST INFRASTRUCTURE ONLY (see keto_oracle.h for the contract
 * and the reference functions restated here, with file:line citations).
 *
 * Deliberately simple: rows live in one table sorted by the reference's ORDER BY,
 * every "SQL query" is a binary-searched range plus a residual filter, every page
 * goes through the same string-level namespace lookups as toInternal, and the
 * visited set is a hash set of Subject.String() keys exactly as in graph_utils.go.
 */
#define _GNU_SOURCE
#include "keto_oracle.h"

#include <pthread.h>
#include <time.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ storage */
typedef struct {
    int32_t id;
    char *name;
} ko_ns;

typedef struct {
    int32_t ns_id, ss_ns;
    uint64_t obj, rel, sid, ss_obj, ss_rel; /* arena offsets */
    int64_t ct;
    uint64_t seq;
    uint8_t kind; /* KO_SUBJECT_ID / KO_SUBJECT_SET */
} ko_row;

struct ko_store {
    ko_ns *ns;
    size_t nns, cap_ns;
    ko_row *rows;
    size_t nrows, cap_rows;
    char *arena;
    size_t arena_len, arena_cap;
    int page_size;
    int nulls_last; /* Postgres ORDER BY: NULLs sort last (subject-set rows after subject ids) */
    int finalized;
};

#define STR(s, off) ((s)->arena + (off))

static int grow(void **p, size_t *cap, size_t need, size_t elem) {
    if (need <= *cap) return 0;
    size_t nc = *cap ? *cap : 16;
    while (nc < need) nc *= 2;
    void *q = realloc(*p, nc * elem);
    if (!q) return KO_ENOMEM;
    *p = q;
    *cap = nc;
    return 0;
}

static int arena_put(ko_store *s, const char *str, size_t len, uint64_t *off) {
    if (grow((void **)&s->arena, &s->arena_cap, s->arena_len + len + 1, 1)) return KO_ENOMEM;
    memcpy(s->arena + s->arena_len, str, len);
    s->arena[s->arena_len + len] = 0;
    *off = s->arena_len;
    s->arena_len += len + 1;
    return 0;
}

ko_store *ko_store_new(void) {
    ko_store *s = (ko_store *)calloc(1, sizeof(ko_store));
    if (!s) return NULL;
    s->page_size = 100; /* defaultPageSize, persister.go:45-47 */
    uint64_t dummy;
    arena_put(s, "", 0, &dummy); /* offset 0 = "" */
    return s;
}

void ko_store_free(ko_store *s) {
    if (!s) return;
    for (size_t i = 0; i < s->nns; i++) free(s->ns[i].name);
    free(s->ns);
    free(s->rows);
    free(s->arena);
    free(s);
}

void ko_free(void *p) { free(p); }

int ko_add_namespace(ko_store *s, int32_t id, const char *name) {
    if (grow((void **)&s->ns, &s->cap_ns, s->nns + 1, sizeof(ko_ns))) return KO_ENOMEM;
    s->ns[s->nns].id = id;
    s->ns[s->nns].name = strdup(name ? name : "");
    s->nns++;
    return KO_OK;
}

void ko_set_page_size(ko_store *s, int page_size) { s->page_size = page_size > 0 ? page_size : 100; }
void ko_set_nulls_last(ko_store *s, int nulls_last) { s->nulls_last = nulls_last != 0; }

static int add_row_len(ko_store *s, int32_t nsid, const char *obj, size_t lobj, const char *rel,
                       size_t lrel, int kind, const char *sid, size_t lsid, int32_t ssns,
                       const char *ssobj, size_t lssobj, const char *ssrel, size_t lssrel, int64_t ct) {
    if (grow((void **)&s->rows, &s->cap_rows, s->nrows + 1, sizeof(ko_row))) return KO_ENOMEM;
    ko_row r;
    memset(&r, 0, sizeof r);
    r.ns_id = nsid;
    r.kind = (uint8_t)kind;
    r.ct = ct;
    r.seq = s->nrows;
    if (arena_put(s, obj, lobj, &r.obj) || arena_put(s, rel, lrel, &r.rel)) return KO_ENOMEM;
    if (kind == KO_SUBJECT_ID) {
        if (arena_put(s, sid, lsid, &r.sid)) return KO_ENOMEM;
    } else {
        r.ss_ns = ssns;
        if (arena_put(s, ssobj, lssobj, &r.ss_obj) || arena_put(s, ssrel, lssrel, &r.ss_rel))
            return KO_ENOMEM;
    }
    s->rows[s->nrows++] = r;
    s->finalized = 0;
    return KO_OK;
}

int ko_add_row(ko_store *s, int32_t namespace_id, const char *object, const char *relation,
               const char *subject_id, int32_t ss_namespace_id, const char *ss_object,
               const char *ss_relation, int64_t commit_time) {
    if (subject_id)
        return add_row_len(s, namespace_id, object, strlen(object), relation, strlen(relation),
                           KO_SUBJECT_ID, subject_id, strlen(subject_id), 0, "", 0, "", 0, commit_time);
    return add_row_len(s, namespace_id, object, strlen(object), relation, strlen(relation),
                       KO_SUBJECT_SET, "", 0, ss_namespace_id, ss_object, strlen(ss_object),
                       ss_relation, strlen(ss_relation), commit_time);
}

int ko_add_rows_columnar(ko_store *s, size_t n, const int32_t *namespace_id,
                         const char *object_data, const uint64_t *object_off,
                         const char *relation_data, const uint64_t *relation_off,
                         const uint8_t *subject_kind, const char *subject_id_data,
                         const uint64_t *subject_id_off, const int32_t *ss_namespace_id,
                         const char *ss_object_data, const uint64_t *ss_object_off,
                         const char *ss_relation_data, const uint64_t *ss_relation_off,
                         const int64_t *commit_time) {
    if (grow((void **)&s->rows, &s->cap_rows, s->nrows + n, sizeof(ko_row))) return KO_ENOMEM;
    /* the batch's strings in one arena growth (no doubling copies at 10^9 rows) */
    size_t bytes = 5 * n + object_off[n] - object_off[0] + relation_off[n] - relation_off[0] +
                   subject_id_off[n] - subject_id_off[0] + ss_object_off[n] - ss_object_off[0] +
                   ss_relation_off[n] - ss_relation_off[0];
    if (s->arena_len + bytes > s->arena_cap) {
        char *q = (char *)realloc(s->arena, s->arena_len + bytes);
        if (!q) return KO_ENOMEM;
        s->arena = q;
        s->arena_cap = s->arena_len + bytes;
    }
    for (size_t i = 0; i < n; i++) {
        int kind = subject_kind[i] ? KO_SUBJECT_SET : KO_SUBJECT_ID;
        int rc = add_row_len(
            s, namespace_id[i], object_data + object_off[i], object_off[i + 1] - object_off[i],
            relation_data + relation_off[i], relation_off[i + 1] - relation_off[i], kind,
            subject_id_data + subject_id_off[i], subject_id_off[i + 1] - subject_id_off[i],
            ss_namespace_id ? ss_namespace_id[i] : 0, ss_object_data + ss_object_off[i],
            ss_object_off[i + 1] - ss_object_off[i], ss_relation_data + ss_relation_off[i],
            ss_relation_off[i + 1] - ss_relation_off[i], commit_time ? commit_time[i] : (int64_t)i);
        if (rc) return rc;
    }
    return KO_OK;
}

/* ORDER BY nid, namespace_id, object, relation, subject_id, subject_set_namespace_id,
 *          subject_set_object, subject_set_relation, commit_time
 * (relationtuples.go:215) with SQLite semantics: NULLs sort first, TEXT uses BINARY
 * collation (memcmp, shorter prefix first), INTEGER numerically.  A subject-set row has
 * subject_id NULL, a subject-id row has all subject_set_* NULL.  Ties keep insertion order.
 * With nulls_last (Postgres ASC order under the "C" collation) NULLs sort last instead,
 * which only moves a group's subject-set rows after its subject-id rows. */
static int cmp_rows(const ko_store *s, const ko_row *a, const ko_row *b) {
    int c;
    if (a->ns_id != b->ns_id) return a->ns_id < b->ns_id ? -1 : 1;
    if ((c = strcmp(STR(s, a->obj), STR(s, b->obj)))) return c;
    if ((c = strcmp(STR(s, a->rel), STR(s, b->rel)))) return c;
    if (a->kind != b->kind) /* the NULL subject_id of a subject-set row */
        return (a->kind == KO_SUBJECT_SET) != (s->nulls_last != 0) ? -1 : 1;
    if (a->kind == KO_SUBJECT_ID) {
        if ((c = strcmp(STR(s, a->sid), STR(s, b->sid)))) return c;
    } else {
        if (a->ss_ns != b->ss_ns) return a->ss_ns < b->ss_ns ? -1 : 1;
        if ((c = strcmp(STR(s, a->ss_obj), STR(s, b->ss_obj)))) return c;
        if ((c = strcmp(STR(s, a->ss_rel), STR(s, b->ss_rel)))) return c;
    }
    if (a->ct != b->ct) return a->ct < b->ct ? -1 : 1;
    return 0;
}

static int cmp_rows_stable(const void *x, const void *y, void *arg) {
    const ko_store *s = (const ko_store *)arg;
    const ko_row *a = (const ko_row *)x, *b = (const ko_row *)y;
    int c = cmp_rows(s, a, b);
    if (c) return c;
    return a->seq < b->seq ? -1 : (a->seq > b->seq);
}

int ko_finalize(ko_store *s, int presorted) {
    if (presorted) {
        for (size_t i = 1; i < s->nrows; i++)
            if (cmp_rows(s, &s->rows[i - 1], &s->rows[i]) > 0) return KO_EINVAL;
    } else {
        qsort_r(s->rows, s->nrows, sizeof(ko_row), cmp_rows_stable, s);
    }
    s->finalized = 1;
    return KO_OK;
}

size_t ko_num_rows(const ko_store *s) { return s->nrows; }

/* --------------------------------------------------------- namespace manager */
/* memoryNamespaceManager: linear scan, first match, herodot.ErrNotFound otherwise
 * (internal/driver/config/namespace_memory.go:29-47) */
static const ko_ns *ns_by_name(const ko_store *s, const char *name) {
    for (size_t i = 0; i < s->nns; i++)
        if (!strcmp(s->ns[i].name, name)) return &s->ns[i];
    return NULL;
}
static const ko_ns *ns_by_id(const ko_store *s, int32_t id) {
    for (size_t i = 0; i < s->nns; i++)
        if (s->ns[i].id == id) return &s->ns[i];
    return NULL;
}

/* ---------------------------------------------------------------- subjects */
typedef struct {
    int kind;
    const char *id, *ns, *obj, *rel;
} ko_subj;

/* Subject.String(): SubjectID -> ID, SubjectSet -> "ns:obj#rel" (definitions.go:164-170) */
static size_t subj_key(const ko_subj *x, char **buf, size_t *cap) {
    size_t need;
    if (x->kind == KO_SUBJECT_ID)
        need = strlen(x->id);
    else
        need = strlen(x->ns) + strlen(x->obj) + strlen(x->rel) + 2;
    if (need + 1 > *cap) {
        *cap = (need + 1) * 2;
        *buf = (char *)realloc(*buf, *cap);
    }
    if (x->kind == KO_SUBJECT_ID)
        memcpy(*buf, x->id, need + 1);
    else
        snprintf(*buf, need + 1, "%s:%s#%s", x->ns, x->obj, x->rel);
    return need;
}

/* typed equality (definitions.go:253-267) */
static int subj_equals(const ko_subj *a, const ko_subj *b) {
    if (a->kind != b->kind) return 0;
    if (a->kind == KO_SUBJECT_ID) return !strcmp(a->id, b->id);
    return !strcmp(a->rel, b->rel) && !strcmp(a->obj, b->obj) && !strcmp(a->ns, b->ns);
}

/* ------------------------------------------------------ visited string set */
typedef struct {
    uint64_t *h;   /* hash per slot (0 = empty) */
    size_t *off;   /* key offset in keys */
    size_t cap, n;
    char *keys;
    size_t klen, kcap;
} kset;

static uint64_t fnv(const char *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
    return h | 1;
}

static kset *kset_new(void) {
    kset *k = (kset *)calloc(1, sizeof(kset));
    k->cap = 16;
    k->h = (uint64_t *)calloc(k->cap, sizeof(uint64_t));
    k->off = (size_t *)calloc(k->cap, sizeof(size_t));
    return k;
}
static void kset_free(kset *k) {
    if (!k) return;
    free(k->h);
    free(k->off);
    free(k->keys);
    free(k);
}
static void kset_rehash(kset *k) {
    size_t oc = k->cap;
    uint64_t *oh = k->h;
    size_t *oo = k->off;
    k->cap *= 2;
    k->h = (uint64_t *)calloc(k->cap, sizeof(uint64_t));
    k->off = (size_t *)calloc(k->cap, sizeof(size_t));
    for (size_t i = 0; i < oc; i++)
        if (oh[i]) {
            size_t j = oh[i] & (k->cap - 1);
            while (k->h[j]) j = (j + 1) & (k->cap - 1);
            k->h[j] = oh[i];
            k->off[j] = oo[i];
        }
    free(oh);
    free(oo);
}
/* returns 1 if key was already present, else inserts and returns 0 */
static int kset_test_add(kset *k, const char *key, size_t len) {
    uint64_t h = fnv(key, len);
    size_t j = h & (k->cap - 1);
    while (k->h[j]) {
        if (k->h[j] == h && !strcmp(k->keys + k->off[j], key)) return 1;
        j = (j + 1) & (k->cap - 1);
    }
    if (k->klen + len + 1 > k->kcap) {
        k->kcap = (k->klen + len + 1) * 2;
        k->keys = (char *)realloc(k->keys, k->kcap);
    }
    memcpy(k->keys + k->klen, key, len + 1);
    k->h[j] = h;
    k->off[j] = k->klen;
    k->klen += len + 1;
    if (++k->n * 2 > k->cap) kset_rehash(k);
    return 0;
}

/* ------------------------------------------------------ GetRelationTuples */
typedef struct {
    const char *ns, *obj, *rel; /* "" = no filter (relationtuples.go:218-236) */
} ko_query;

typedef struct {
    ko_subj *subj;
    size_t n, cap;
    int has_next;
} ko_page;

static size_t lb_ns(const ko_store *s, size_t lo, size_t hi, int32_t id, int upper) {
    while (lo < hi) {
        size_t m = lo + (hi - lo) / 2;
        int32_t v = s->rows[m].ns_id;
        if (upper ? v <= id : v < id)
            lo = m + 1;
        else
            hi = m;
    }
    return lo;
}
static size_t lb_str(const ko_store *s, size_t lo, size_t hi, int field, const char *key, int upper) {
    while (lo < hi) {
        size_t m = lo + (hi - lo) / 2;
        const char *v = STR(s, field == 0 ? s->rows[m].obj : s->rows[m].rel);
        int c = strcmp(v, key);
        if (upper ? c <= 0 : c < 0)
            lo = m + 1;
        else
            hi = m;
    }
    return lo;
}

static int row_matches(const ko_store *s, const ko_row *r, int have_ns, int32_t nsid, const ko_query *q) {
    if (have_ns && r->ns_id != nsid) return 0;
    if (q->obj[0] && strcmp(STR(s, r->obj), q->obj)) return 0;
    if (q->rel[0] && strcmp(STR(s, r->rel), q->rel)) return 0;
    return 1;
}

/* one page (1-based) of the filtered, ordered result, converted with toInternal */
static int get_page(const ko_store *s, const ko_query *q, int page, ko_page *out) {
    out->n = 0;
    out->has_next = 0;
    int have_ns = q->ns[0] != 0;
    int32_t nsid = 0;
    if (have_ns) {
        const ko_ns *n = ns_by_name(s, q->ns);
        if (!n) return KO_ENOTFOUND; /* relationtuples.go:230-236 */
        nsid = n->id;
    }
    /* narrow along the ORDER BY prefix, then filter the residual */
    size_t lo = 0, hi = s->nrows;
    int residual = 0;
    if (have_ns) {
        size_t a = lb_ns(s, lo, hi, nsid, 0), b = lb_ns(s, lo, hi, nsid, 1);
        lo = a;
        hi = b;
        if (q->obj[0]) {
            a = lb_str(s, lo, hi, 0, q->obj, 0);
            b = lb_str(s, lo, hi, 0, q->obj, 1);
            lo = a;
            hi = b;
            if (q->rel[0]) {
                a = lb_str(s, lo, hi, 1, q->rel, 0);
                b = lb_str(s, lo, hi, 1, q->rel, 1);
                lo = a;
                hi = b;
            }
        } else if (q->rel[0])
            residual = 1;
    } else if (q->obj[0] || q->rel[0])
        residual = 1;

    size_t ps = (size_t)s->page_size, first = (size_t)(page - 1) * ps;
    size_t total = 0;
    const ko_row **sel = NULL;
    size_t nsel = 0;
    if (!residual) {
        total = hi - lo;
        size_t b = lo + first, e = lo + first + ps;
        if (b > hi) b = hi;
        if (e > hi) e = hi;
        nsel = e - b;
        sel = (const ko_row **)malloc((nsel ? nsel : 1) * sizeof(*sel));
        for (size_t i = 0; i < nsel; i++) sel[i] = &s->rows[b + i];
    } else {
        sel = (const ko_row **)malloc(ps * sizeof(*sel));
        for (size_t i = lo; i < hi; i++)
            if (row_matches(s, &s->rows[i], have_ns, nsid, q)) {
                if (total >= first && total < first + ps) sel[nsel++] = &s->rows[i];
                total++;
            }
    }
    /* next token unless Page >= TotalPages (relationtuples.go:243-246) */
    size_t total_pages = (total + ps - 1) / ps;
    out->has_next = (size_t)page < total_pages;
    /* toInternal for every row of the page; any failure fails the page (:248-255) */
    if (nsel > out->cap) {
        out->cap = nsel;
        out->subj = (ko_subj *)realloc(out->subj, nsel * sizeof(ko_subj));
    }
    for (size_t i = 0; i < nsel; i++) {
        const ko_row *r = sel[i];
        if (!ns_by_id(s, r->ns_id)) {
            free(sel);
            return KO_ENOTFOUND;
        }
        ko_subj *x = &out->subj[i];
        x->kind = r->kind;
        if (r->kind == KO_SUBJECT_ID) {
            x->id = STR(s, r->sid);
            x->ns = x->obj = x->rel = "";
        } else {
            const ko_ns *n = ns_by_id(s, r->ss_ns);
            if (!n) {
                free(sel);
                return KO_ENOTFOUND;
            }
            x->id = "";
            x->ns = n->name;
            x->obj = STR(s, r->ss_obj);
            x->rel = STR(s, r->ss_rel);
        }
    }
    out->n = nsel;
    free(sel);
    return KO_OK;
}

/* -------------------------------------------------------------------- check */
typedef struct {
    const ko_store *s;
    const ko_subj *req;
    char *kbuf;
    size_t kcap;
    double deadline; /* CLOCK_MONOTONIC seconds; 0 = none (ko_check_batch_budget) */
    unsigned tick;
} chk_ctx;

static double mono_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

static int check_one_further(chk_ctx *c, kset *visited, const ko_query *q);

/* subjectIsAllowed (internal/check/engine.go:33-67).  `visited` == NULL models a ctx
 * without a visited map: CheckAndAddVisited then creates a FRESH map holding only this
 * subject, and the loop-scoped ctx (engine.go:40) carries it into this tuple's subtree
 * only. */
static int subject_is_allowed(chk_ctx *c, kset *visited, const ko_page *rels) {
    for (size_t i = 0; i < rels->n; i++) {
        const ko_subj *sr = &rels->subj[i];
        size_t klen = subj_key(sr, &c->kbuf, &c->kcap);
        kset *child = visited, *fresh = NULL;
        if (!visited) {
            fresh = child = kset_new();
            kset_test_add(fresh, c->kbuf, klen);
        } else if (kset_test_add(visited, c->kbuf, klen)) {
            continue; /* wasAlreadyVisited */
        }
        if (subj_equals(c->req, sr)) {
            kset_free(fresh);
            return 1;
        }
        if (sr->kind != KO_SUBJECT_SET) {
            kset_free(fresh);
            continue;
        }
        ko_query q = {sr->ns, sr->obj, sr->rel};
        int r = check_one_further(c, child, &q);
        kset_free(fresh);
        if (r) return r; /* allowed (1) or error (<0) */
    }
    return 0;
}

/* checkOneIndirectionFurther (internal/check/engine.go:69-91) */
static int check_one_further(chk_ctx *c, kset *visited, const ko_query *q) {
    /* a per-request time budget (test harness only: the reference has none) */
    if (c->deadline > 0 && !(++c->tick & 255) && mono_s() > c->deadline) return KO_ETIMEOUT;
    ko_page pg = {0};
    int rc = 0;
    for (int page = 1;; page++) {
        int e = get_page(c->s, q, page, &pg);
        if (e == KO_ENOTFOUND) {
            rc = 0; /* herodot.ErrNotFound -> false */
            break;
        }
        if (e) {
            rc = e;
            break;
        }
        /* rows of one page are consumed before the next page is fetched */
        int r = subject_is_allowed(c, visited, &pg);
        if (r || !pg.has_next) {
            rc = r;
            break;
        }
    }
    free(pg.subj);
    return rc;
}

static int make_subj(int kind, const char *sid, const char *sns, const char *sobj, const char *srel,
                     ko_subj *out) {
    if (kind == KO_SUBJECT_ID) {
        out->kind = KO_SUBJECT_ID;
        out->id = sid ? sid : "";
        out->ns = out->obj = out->rel = "";
        return KO_OK;
    }
    if (kind == KO_SUBJECT_SET) {
        out->kind = KO_SUBJECT_SET;
        out->id = "";
        out->ns = sns ? sns : "";
        out->obj = sobj ? sobj : "";
        out->rel = srel ? srel : "";
        return KO_OK;
    }
    return KO_EINVAL; /* nil subject: relationtuple.ErrNilSubject */
}

static int check_budget(const ko_store *s, const char *ns, const char *obj, const char *rel, int subject_kind,
                        const char *subject_id, const char *ss_ns, const char *ss_obj, const char *ss_rel,
                        double seconds, int *allowed) {
    *allowed = 0;
    if (!s->finalized) return KO_EINVAL;
    ko_subj req;
    int e = make_subj(subject_kind, subject_id, ss_ns, ss_obj, ss_rel, &req);
    if (e) return e;
    chk_ctx c = {s, &req, NULL, 0, seconds > 0 ? mono_s() + seconds : 0, 0};
    ko_query q = {ns ? ns : "", obj ? obj : "", rel ? rel : ""};
    int r = check_one_further(&c, NULL, &q); /* SubjectIsAllowed, engine.go:93-95 */
    free(c.kbuf);
    if (r < 0) return r;
    *allowed = r;
    return KO_OK;
}

int ko_check(const ko_store *s, const char *ns, const char *obj, const char *rel, int subject_kind,
             const char *subject_id, const char *ss_ns, const char *ss_obj, const char *ss_rel,
             int *allowed) {
    return check_budget(s, ns, obj, rel, subject_kind, subject_id, ss_ns, ss_obj, ss_rel, 0, allowed);
}

typedef struct {
    const ko_store *s;
    size_t n;
    const char *const *ns, *const *obj, *const *rel, *const *sid, *const *sns, *const *sobj,
        *const *srel;
    const int *kind;
    uint8_t *allowed;
    int *status;
    double budget; /* seconds per request, 0 = none */
    atomic_size_t next;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 1);
        if (i >= j->n) break;
        int a = 0;
        j->status[i] = check_budget(j->s, j->ns[i], j->obj[i], j->rel[i], j->kind[i], j->sid ? j->sid[i] : NULL,
                                    j->sns ? j->sns[i] : NULL, j->sobj ? j->sobj[i] : NULL,
                                    j->srel ? j->srel[i] : NULL, j->budget, &a);
        j->allowed[i] = (uint8_t)a;
    }
    return NULL;
}

int ko_check_batch(const ko_store *s, size_t n, const char *const *ns, const char *const *obj,
                   const char *const *rel, const int *subject_kind, const char *const *subject_id,
                   const char *const *ss_ns, const char *const *ss_obj, const char *const *ss_rel,
                   int nthreads, uint8_t *allowed, int *status) {
    return ko_check_batch_budget(s, n, ns, obj, rel, subject_kind, subject_id, ss_ns, ss_obj, ss_rel, nthreads, 0,
                                 allowed, status);
}

int ko_check_batch_budget(const ko_store *s, size_t n, const char *const *ns, const char *const *obj,
                          const char *const *rel, const int *subject_kind, const char *const *subject_id,
                          const char *const *ss_ns, const char *const *ss_obj, const char *const *ss_rel,
                          int nthreads, double seconds_per_request, uint8_t *allowed, int *status) {
    batch_job j;
    memset(&j, 0, sizeof j);
    j.budget = seconds_per_request;
    j.s = s; j.n = n; j.ns = ns; j.obj = obj; j.rel = rel; j.sid = subject_id; j.sns = ss_ns;
    j.sobj = ss_obj; j.srel = ss_rel; j.kind = subject_kind; j.allowed = allowed; j.status = status;
    atomic_init(&j.next, 0);
    if (nthreads < 1) nthreads = 1;
    pthread_t *t = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, (size_t)256 << 20); /* deep recursion, like Go's growable stacks */
    for (int i = 0; i < nthreads; i++) pthread_create(&t[i], &attr, batch_worker, &j);
    for (int i = 0; i < nthreads; i++) pthread_join(t[i], NULL);
    pthread_attr_destroy(&attr);
    free(t);
    return KO_OK;
}

/* ------------------------------------------------------------------- expand */
enum { T_UNION = 0, T_LEAF = 1 };
typedef struct tnode {
    int type;
    ko_subj subj;
    struct tnode **ch;
    size_t nch, cap;
} tnode;

static tnode *tnode_new(int type, const ko_subj *x) {
    tnode *t = (tnode *)calloc(1, sizeof(tnode));
    t->type = type;
    t->subj = *x;
    return t;
}
static void tnode_free(tnode *t) {
    if (!t) return;
    for (size_t i = 0; i < t->nch; i++) tnode_free(t->ch[i]);
    free(t->ch);
    free(t);
}
static void tnode_push(tnode *t, tnode *c) {
    if (t->nch == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 4;
        t->ch = (tnode **)realloc(t->ch, t->cap * sizeof(tnode *));
    }
    t->ch[t->nch++] = c;
}

typedef struct {
    const ko_store *s;
    kset *visited; /* one map for the whole tree (created by the root call) */
    char *kbuf;
    size_t kcap;
} exp_ctx;

/* BuildTree (internal/expand/engine.go:30-98) */
static int build_tree(exp_ctx *c, const ko_subj *subject, int rest_depth, tnode **out) {
    *out = NULL;
    if (rest_depth <= 0) return KO_OK;
    if (subject->kind != KO_SUBJECT_SET) {
        *out = tnode_new(T_LEAF, subject);
        return KO_OK;
    }
    size_t klen = subj_key(subject, &c->kbuf, &c->kcap);
    if (!c->visited) {
        c->visited = kset_new();
        kset_test_add(c->visited, c->kbuf, klen);
    } else if (kset_test_add(c->visited, c->kbuf, klen)) {
        return KO_OK; /* already visited -> nil */
    }
    tnode *sub = tnode_new(T_UNION, subject);
    ko_query q = {subject->ns, subject->obj, subject->rel};
    ko_page pg = {0};
    int rc = KO_OK;
    for (int page = 1;; page++) {
        int e = get_page(c->s, &q, page, &pg);
        if (e) {
            rc = e;
            tnode_free(sub);
            sub = NULL;
            break;
        }
        if (pg.n == 0) {
            tnode_free(sub);
            sub = NULL;
            break;
        }
        if (rest_depth <= 1) {
            sub->type = T_LEAF;
            break;
        }
        /* the page's subjects must outlive recursion (pg is reused) */
        size_t n = pg.n;
        ko_subj *rows = (ko_subj *)malloc(n * sizeof(ko_subj));
        memcpy(rows, pg.subj, n * sizeof(ko_subj));
        int has_next = pg.has_next;
        for (size_t i = 0; i < n; i++) {
            tnode *child = NULL;
            int e2 = build_tree(c, &rows[i], rest_depth - 1, &child);
            if (e2) {
                rc = e2;
                break;
            }
            if (!child) child = tnode_new(T_LEAF, &rows[i]);
            tnode_push(sub, child);
        }
        free(rows);
        if (rc) {
            tnode_free(sub);
            sub = NULL;
            break;
        }
        if (!has_next) break;
    }
    free(pg.subj);
    *out = sub;
    return rc;
}

/* --------------------------------------------------------------------- JSON */
typedef struct {
    char *p;
    size_t n, cap;
} sbuf;
static void sb_put(sbuf *b, const char *s, size_t n) {
    if (b->n + n + 1 > b->cap) {
        b->cap = (b->n + n + 1) * 2;
        b->p = (char *)realloc(b->p, b->cap);
    }
    memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void sb_cstr(sbuf *b, const char *s) { sb_put(b, s, strlen(s)); }
static void sb_jstr(sbuf *b, const char *s) {
    sb_put(b, "\"", 1);
    for (const unsigned char *p = (const unsigned char *)s; *p; p++) {
        char tmp[8];
        if (*p == '"' || *p == '\\') {
            tmp[0] = '\\';
            tmp[1] = (char)*p;
            sb_put(b, tmp, 2);
        } else if (*p < 0x20) {
            snprintf(tmp, sizeof tmp, "\\u%04x", *p);
            sb_put(b, tmp, 6);
        } else
            sb_put(b, (const char *)p, 1);
    }
    sb_put(b, "\"", 1);
}
static void sb_subject_fields(sbuf *b, const ko_subj *x) {
    if (x->kind == KO_SUBJECT_ID) {
        sb_cstr(b, "\"subject_id\":");
        sb_jstr(b, x->id);
    } else {
        sb_cstr(b, "\"subject_set\":{\"namespace\":");
        sb_jstr(b, x->ns);
        sb_cstr(b, ",\"object\":");
        sb_jstr(b, x->obj);
        sb_cstr(b, ",\"relation\":");
        sb_jstr(b, x->rel);
        sb_cstr(b, "}");
    }
}
/* node{type, children omitempty, subject_id, subject_set} (tree.go:85-91) */
static void sb_tree(sbuf *b, const tnode *t) {
    sb_cstr(b, t->type == T_UNION ? "{\"type\":\"union\"," : "{\"type\":\"leaf\",");
    if (t->nch) {
        sb_cstr(b, "\"children\":[");
        for (size_t i = 0; i < t->nch; i++) {
            if (i) sb_cstr(b, ",");
            sb_tree(b, t->ch[i]);
        }
        sb_cstr(b, "],");
    }
    sb_subject_fields(b, &t->subj);
    sb_cstr(b, "}");
}

int ko_expand(const ko_store *s, int subject_kind, const char *subject_id, const char *ss_ns,
              const char *ss_obj, const char *ss_rel, int rest_depth, char **json) {
    *json = NULL;
    if (!s->finalized) return KO_EINVAL;
    ko_subj subj;
    int e = make_subj(subject_kind, subject_id, ss_ns, ss_obj, ss_rel, &subj);
    if (e) return e;
    exp_ctx c = {s, NULL, NULL, 0};
    tnode *t = NULL;
    e = build_tree(&c, &subj, rest_depth, &t);
    kset_free(c.visited);
    free(c.kbuf);
    if (e) {
        tnode_free(t);
        return e;
    }
    sbuf b = {0};
    if (!t)
        sb_cstr(&b, "null");
    else
        sb_tree(&b, t);
    tnode_free(t);
    *json = b.p;
    return KO_OK;
}

int ko_get_page(const ko_store *s, const char *ns, const char *obj, const char *rel, int page,
                char **json, int *has_next) {
    *json = NULL;
    *has_next = 0;
    if (!s->finalized || page < 1) return KO_EINVAL;
    ko_query q = {ns ? ns : "", obj ? obj : "", rel ? rel : ""};
    ko_page pg = {0};
    int e = get_page(s, &q, page, &pg);
    if (e) {
        free(pg.subj);
        return e;
    }
    /* report the owner fields too: re-run the selection to know them is unnecessary
     * for ordering tests, which compare subjects in order */
    sbuf b = {0};
    sb_cstr(&b, "[");
    for (size_t i = 0; i < pg.n; i++) {
        if (i) sb_cstr(&b, ",");
        sb_cstr(&b, "{");
        sb_subject_fields(&b, &pg.subj[i]);
        sb_cstr(&b, "}");
    }
    sb_cstr(&b, "]");
    *has_next = pg.has_next;
    free(pg.subj);
    *json = b.p;
    return KO_OK;
}
