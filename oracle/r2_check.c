/*
 * r2_check — TEST INFRASTRUCTURE ONLY: an independent checker of the R2 reachability
 * formula for graphs too large for the reference's DFS (keto_oracle.c) to finish.
 *
 * The reference (internal/check/engine.go:33-95) answers, when no two typed subjects
 * share a String() key (R4), "is the requested subject S the subject of some tuple
 * reachable from the root group through >= 1 tuple" (SURVEY.md 8.0 R2):
 *
 *     allowed(r, t)  <=>  r in P(t)  or  P(t) ∩ X(r) != {}
 *
 * with P(t) = the groups having a tuple whose subject is t, and X(r) = the subject sets
 * reachable from r along subject-set tuples (a subject set (ns, obj, rel) expands into
 * the rows of the group (ns, obj, rel), engine.go:57; typed equality, definitions.go:
 * 253-267).  This file shares NO code with libketogpu: it interns the raw row stream
 * itself (typed keys, full byte compare), builds its own adjacency, and evaluates X(r)
 * by a multi-source bitset BFS (64 requests per 64-bit word, one word per task, worker
 * threads) — so a bug in the snapshot layer, its node numbering or the device record
 * layout cannot pass both the engine and this check.
 *
 * Scope (checked, else refused): every namespace id of the rows is configured (no page
 * poisoning, R7), no subject set has an empty field (no R5 wildcards), roots have no empty
 * field.  An unknown root namespace name answers false (R6, engine.go:75-77).  R4 is the
 * caller's precondition (the scale graphs' snapshots report no shared keys).
 * Pinned by tests/test_oracle.py against keto_oracle.c on the randgraph, RBAC, folder and
 * power-law fixtures.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "r2_check.h"

/* ------------------------------------------------------------ typed key interning */
typedef struct {
    uint64_t *hash; /* slot -> hash (0 = empty) */
    uint32_t *id;   /* slot -> node id */
    size_t cap;
    char *arena; /* key bytes of node i at arena[off[i] .. off[i+1]) */
    size_t arena_n, arena_cap;
    uint64_t *off;
    size_t n, off_cap;
} intern_t;

static uint64_t fnv(const char *p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; i++) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
    return h;
}

/* key of a subject set / group: ns id, object, relation (typed: a SubjectID never equals
 * a SubjectSet, and the two kinds are interned in separate tables) */
static size_t set_key(char *buf, int32_t ns, const char *o, size_t on, const char *r, size_t rn) {
    memcpy(buf, &ns, 4);
    uint32_t on32 = (uint32_t)on;
    memcpy(buf + 4, &on32, 4);
    memcpy(buf + 8, o, on);
    memcpy(buf + 8 + on, r, rn);
    return 8 + on + rn;
}

static int grow(intern_t *t) {
    const size_t ncap = t->cap ? 2 * t->cap : 1 << 16;
    uint64_t *h = calloc(ncap, 8);
    uint32_t *id = malloc(ncap * 4);
    if (!h || !id) return -1;
    for (size_t i = 0; i < t->cap; i++)
        if (t->hash[i]) {
            size_t j = t->hash[i] & (ncap - 1);
            while (h[j]) j = (j + 1) & (ncap - 1);
            h[j] = t->hash[i];
            id[j] = t->id[i];
        }
    free(t->hash);
    free(t->id);
    t->hash = h;
    t->id = id;
    t->cap = ncap;
    return 0;
}

/* id of key (inserted when absent and insert != 0); UINT32_MAX when absent */
static uint32_t intern(intern_t *t, const char *k, size_t n, int insert) {
    if (insert && 2 * (t->n + 1) > t->cap && grow(t)) return UINT32_MAX - 1;
    if (!t->cap) return UINT32_MAX;
    const uint64_t h = fnv(k, n, 1469598103934665603ull) | 1;
    size_t j = h & (t->cap - 1);
    while (t->hash[j]) {
        if (t->hash[j] == h) {
            const uint32_t i = t->id[j];
            if (t->off[i + 1] - t->off[i] == n && !memcmp(t->arena + t->off[i], k, n)) return i;
        }
        j = (j + 1) & (t->cap - 1);
    }
    if (!insert) return UINT32_MAX;
    if (t->arena_n + n > t->arena_cap) {
        size_t c = t->arena_cap ? 2 * t->arena_cap : 1 << 20;
        while (c < t->arena_n + n) c *= 2;
        char *a = realloc(t->arena, c);
        if (!a) return UINT32_MAX - 1;
        t->arena = a;
        t->arena_cap = c;
    }
    if (t->n + 2 > t->off_cap) {
        size_t c = t->off_cap ? 2 * t->off_cap : 1 << 16;
        uint64_t *o = realloc(t->off, c * 8);
        if (!o) return UINT32_MAX - 1;
        t->off = o;
        t->off_cap = c;
        if (!t->n) t->off[0] = 0;
    }
    memcpy(t->arena + t->arena_n, k, n);
    t->arena_n += n;
    const uint32_t id = (uint32_t)t->n++;
    t->off[id + 1] = t->arena_n;
    t->hash[j] = h;
    t->id[j] = id;
    return id;
}

static void intern_free(intern_t *t) {
    free(t->hash);
    free(t->id);
    free(t->arena);
    free(t->off);
}

/* ------------------------------------------------------------------------ state */
typedef struct {
    uint32_t a, b;
} pair_t;

struct kr_checker {
    int32_t *ns_id;
    char **ns_name;
    size_t nns;
    intern_t sets;  /* subject sets / groups */
    intern_t sids;  /* the requests' subject-id targets only */
    size_t n;       /* requests */
    uint32_t *root; /* set node, or UINT32_MAX (unknown namespace: false) */
    uint32_t *tgt;  /* target key: set node, or sid key | 1<<31 (UINT32_MAX: never equal) */
    int *status;
    uint8_t *is_target_set; /* per set node (grown lazily) */
    size_t is_target_cap;
    pair_t *edge; /* (group, subject set) */
    size_t ne, ne_cap;
    pair_t *par; /* (target key, group): a row of the group has the target as subject */
    size_t np, np_cap;
    int32_t last_ns; /* the previous row's group (rows arrive grouped) */
    const char *last_o, *last_r;
    size_t last_on, last_rn;
    uint32_t last_g;
    /* finished */
    uint64_t *csr_off;
    uint32_t *csr_col;
    uint64_t *p_off; /* per request: its P(t) groups, from the sorted pairs */
    uint32_t *p_col;
    int finished;
    char err[256];
};

static const int32_t *ns_lookup_name(const kr_checker *k, const char *name) { /* first match */
    for (size_t i = 0; i < k->nns; i++)
        if (!strcmp(k->ns_name[i], name)) return &k->ns_id[i];
    return NULL;
}
static int ns_known(const kr_checker *k, int32_t id) {
    for (size_t i = 0; i < k->nns; i++)
        if (k->ns_id[i] == id) return 1;
    return 0;
}

kr_checker *kr_new(const int32_t *ids, const char *const *names, size_t nns) {
    kr_checker *k = calloc(1, sizeof *k);
    k->ns_id = malloc((nns + 1) * sizeof *k->ns_id);
    k->ns_name = malloc((nns + 1) * sizeof *k->ns_name);
    for (size_t i = 0; i < nns; i++) k->ns_id[i] = ids[i], k->ns_name[i] = strdup(names[i]);
    k->nns = nns;
    k->last_g = UINT32_MAX;
    return k;
}

const char *kr_error(const kr_checker *k) { return k->err; }

static int push_pair(pair_t **v, size_t *n, size_t *cap, uint32_t a, uint32_t b) {
    if (*n == *cap) {
        size_t c = *cap ? 2 * *cap : 1 << 16;
        pair_t *p = realloc(*v, c * sizeof *p);
        if (!p) return -1;
        *v = p;
        *cap = c;
    }
    (*v)[(*n)++] = (pair_t){a, b};
    return 0;
}

static void mark_target(kr_checker *k, uint32_t v) {
    if (v >= k->is_target_cap) {
        size_t c = k->is_target_cap ? k->is_target_cap : 1024;
        while (c <= v) c *= 2;
        k->is_target_set = realloc(k->is_target_set, c);
        memset(k->is_target_set + k->is_target_cap, 0, c - k->is_target_cap);
        k->is_target_cap = c;
    }
    k->is_target_set[v] = 1;
}

int kr_add_requests(kr_checker *k, size_t n, const char *const *ns, const char *const *obj, const char *const *rel,
                    const int *kind, const char *const *sid, const char *const *ss_ns, const char *const *ss_obj,
                    const char *const *ss_rel) {
    char buf[8 + 2 * 4096];
    k->n = n;
    k->root = malloc(n * 4);
    k->tgt = malloc(n * 4);
    k->status = calloc(n, sizeof(int));
    for (size_t i = 0; i < n; i++) {
        k->root[i] = k->tgt[i] = UINT32_MAX;
        const size_t on = strlen(obj[i]), rn = strlen(rel[i]);
        if (!ns[i][0] || !on || !rn || on > 4096 || rn > 4096) { /* R5 wildcard roots: out of scope */
            k->status[i] = KR_EREFUSED;
            continue;
        }
        const int32_t *nid = ns_lookup_name(k, ns[i]);
        if (nid) k->root[i] = intern(&k->sets, buf, set_key(buf, *nid, obj[i], on, rel[i], rn), 1);
        if (kind[i] == 0) {
            const size_t sn = strlen(sid[i]);
            const uint32_t s = intern(&k->sids, sid[i], sn, 1);
            k->tgt[i] = s | 0x80000000u;
        } else if (kind[i] == 1) {
            const size_t so = strlen(ss_obj[i]), sr = strlen(ss_rel[i]);
            const int32_t *sn = ns_lookup_name(k, ss_ns[i]);
            if (sn && so <= 4096 && sr <= 4096) {
                const uint32_t v = intern(&k->sets, buf, set_key(buf, *sn, ss_obj[i], so, ss_rel[i], sr), 1);
                k->tgt[i] = v;
                mark_target(k, v);
            }
        } else {
            k->status[i] = KR_EREFUSED; /* nil subject */
        }
    }
    return KR_OK;
}

int kr_add_rows_columnar(kr_checker *k, size_t n, const int32_t *ns, const char *od, const uint64_t *oo,
                         const char *rd, const uint64_t *ro, const uint8_t *kind, const char *sd, const uint64_t *so,
                         const int32_t *ssns, const char *sod, const uint64_t *soo, const char *srd,
                         const uint64_t *sro) {
    char buf[8 + 2 * 4096];
    for (size_t i = 0; i < n; i++) {
        const char *o = od + oo[i], *r = rd + ro[i];
        const size_t on = oo[i + 1] - oo[i], rn = ro[i + 1] - ro[i];
        if (on > 4096 || rn > 4096) {
            snprintf(k->err, sizeof k->err, "row %zu: field longer than 4096 bytes", i);
            return KR_EREFUSED;
        }
        if (ns[i] != k->last_ns || on != k->last_on || rn != k->last_rn || memcmp(o, k->last_o, on) ||
            memcmp(r, k->last_r, rn)) {
            if (!ns_known(k, ns[i])) {
                snprintf(k->err, sizeof k->err, "row %zu: namespace id %d is not configured (R7 out of scope)", i,
                         ns[i]);
                return KR_EREFUSED;
            }
            k->last_ns = ns[i];
            k->last_o = o;
            k->last_r = r;
            k->last_on = on;
            k->last_rn = rn;
            k->last_g = UINT32_MAX; /* interned on first use */
        }
        uint32_t g = k->last_g;
#define GROUP()                                                                          \
    do {                                                                                 \
        if (g == UINT32_MAX) {                                                           \
            g = k->last_g = intern(&k->sets, buf, set_key(buf, ns[i], o, on, r, rn), 1); \
            if (g >= UINT32_MAX - 1) return KR_ENOMEM;                                   \
        }                                                                                \
    } while (0)
        if (kind[i] == 0) {
            const uint32_t s = intern(&k->sids, sd + so[i], so[i + 1] - so[i], 0);
            if (s != UINT32_MAX) {
                GROUP();
                if (push_pair(&k->par, &k->np, &k->np_cap, s | 0x80000000u, g)) return KR_ENOMEM;
            }
            continue;
        }
        const size_t s_on = soo[i + 1] - soo[i], s_rn = sro[i + 1] - sro[i];
        if (!ns_known(k, ssns[i])) {
            snprintf(k->err, sizeof k->err, "row %zu: subject set namespace id %d is not configured", i, ssns[i]);
            return KR_EREFUSED;
        }
        if (!s_on || !s_rn) {
            snprintf(k->err, sizeof k->err, "row %zu: subject set with an empty field (R5 out of scope)", i);
            return KR_EREFUSED;
        }
        if (s_on > 4096 || s_rn > 4096) return KR_EREFUSED;
        GROUP();
        const uint32_t s = intern(&k->sets, buf, set_key(buf, ssns[i], sod + soo[i], s_on, srd + sro[i], s_rn), 1);
        if (s >= UINT32_MAX - 1) return KR_ENOMEM;
        if (push_pair(&k->edge, &k->ne, &k->ne_cap, g, s)) return KR_ENOMEM;
        if (s < k->is_target_cap && k->is_target_set[s] && push_pair(&k->par, &k->np, &k->np_cap, s, g))
            return KR_ENOMEM;
#undef GROUP
    }
    k->last_o = k->last_r = NULL; /* the caller's buffers end here */
    k->last_on = k->last_rn = (size_t)-1;
    return KR_OK;
}

static int cmp_pair(const void *x, const void *y) {
    const pair_t *a = x, *b = y;
    return a->a < b->a ? -1 : a->a > b->a ? 1 : (a->b < b->b ? -1 : a->b > b->b);
}

int kr_finish(kr_checker *k) {
    const size_t N = k->sets.n;
    /* adjacency of the subject-set graph (counting sort by group) */
    k->csr_off = calloc(N + 1, 8);
    k->csr_col = malloc((k->ne + 1) * 4);
    if (!k->csr_off || !k->csr_col) return KR_ENOMEM;
    for (size_t e = 0; e < k->ne; e++) k->csr_off[k->edge[e].a + 1]++;
    for (size_t v = 0; v < N; v++) k->csr_off[v + 1] += k->csr_off[v];
    uint64_t *cur = malloc((N + 1) * 8);
    memcpy(cur, k->csr_off, (N + 1) * 8);
    for (size_t e = 0; e < k->ne; e++) k->csr_col[cur[k->edge[e].a]++] = k->edge[e].b;
    free(cur);
    free(k->edge);
    k->edge = NULL;
    /* P(t) per request: the parents of its target key */
    qsort(k->par, k->np, sizeof *k->par, cmp_pair);
    k->p_off = calloc(k->n + 1, 8);
    size_t total = 0;
    for (size_t i = 0; i < k->n; i++) {
        pair_t lo = {k->tgt[i], 0};
        size_t a = 0, b = k->np; /* first pair with key >= tgt */
        while (a < b) {
            size_t m = (a + b) / 2;
            if (cmp_pair(&k->par[m], &lo) < 0)
                a = m + 1;
            else
                b = m;
        }
        size_t e = a;
        while (e < k->np && k->par[e].a == k->tgt[i]) e++;
        total += k->tgt[i] == UINT32_MAX ? 0 : e - a;
        k->p_off[i + 1] = total;
    }
    k->p_col = malloc((total + 1) * 4);
    for (size_t i = 0; i < k->n; i++) {
        if (k->tgt[i] == UINT32_MAX) continue;
        pair_t lo = {k->tgt[i], 0};
        size_t a = 0, b = k->np;
        while (a < b) {
            size_t m = (a + b) / 2;
            if (cmp_pair(&k->par[m], &lo) < 0)
                a = m + 1;
            else
                b = m;
        }
        for (uint64_t p = k->p_off[i]; p < k->p_off[i + 1]; p++) k->p_col[p] = k->par[a + (p - k->p_off[i])].b;
    }
    free(k->par);
    k->par = NULL;
    k->finished = 1;
    return KR_OK;
}

/* --------------------------------------------------------------- bitset BFS */
typedef struct {
    kr_checker *k;
    uint8_t *allowed;
    uint64_t *closure; /* NULL, or per request |X(r)| (the interior closure the check walked) */
    atomic_size_t next;
    atomic_ullong visits;
} job_t;

static void *worker(void *arg) {
    job_t *j = arg;
    kr_checker *k = j->k;
    const size_t N = k->sets.n;
    uint64_t *vis = calloc(N + 1, 8), *pend = calloc(N + 1, 8);
    uint32_t *touched = malloc((N + 1) * 4), *front = malloc((N + 1) * 4), *nextf = malloc((N + 1) * 4);
    unsigned long long visits = 0;
    for (;;) {
        const size_t w = atomic_fetch_add(&j->next, 1);
        if (w * 64 >= k->n) break;
        const size_t i0 = w * 64, i1 = i0 + 64 < k->n ? i0 + 64 : k->n;
        size_t nt = 0, nf = 0;
        /* level 1: the roots' own rows */
        for (size_t i = i0; i < i1; i++) {
            if (k->status[i] || k->root[i] == UINT32_MAX) continue;
            const uint64_t bit = 1ull << (i - i0);
            const uint32_t r = k->root[i];
            for (uint64_t e = k->csr_off[r]; e < k->csr_off[r + 1]; e++) {
                const uint32_t c = k->csr_col[e];
                if (vis[c] & bit) continue;
                if (!vis[c]) touched[nt++] = c;
                vis[c] |= bit;
                if (!pend[c]) front[nf++] = c;
                pend[c] |= bit;
            }
        }
        /* X(r): no depth cutoff, until no request gains a node */
        while (nf) {
            size_t nn = 0;
            for (size_t f = 0; f < nf; f++) {
                const uint32_t v = front[f];
                const uint64_t m = pend[v];
                pend[v] = 0;
                for (uint64_t e = k->csr_off[v]; e < k->csr_off[v + 1]; e++) {
                    const uint32_t c = k->csr_col[e];
                    const uint64_t nw = m & ~vis[c];
                    visits++;
                    if (!nw) continue;
                    if (!vis[c]) touched[nt++] = c;
                    vis[c] |= nw;
                    if (!pend[c]) nextf[nn++] = c;
                    pend[c] |= nw;
                }
            }
            uint32_t *t = front;
            front = nextf;
            nextf = t;
            nf = nn;
        }
        for (size_t i = i0; i < i1; i++) {
            if (k->status[i]) continue;
            const uint64_t bit = 1ull << (i - i0);
            uint8_t a = 0;
            for (uint64_t p = k->p_off[i]; p < k->p_off[i + 1] && !a; p++) {
                const uint32_t g = k->p_col[p];
                a = g == k->root[i] || (vis[g] & bit);
            }
            j->allowed[i] = a;
        }
        if (j->closure)
            for (size_t t = 0; t < nt; t++)
                for (uint64_t m = vis[touched[t]]; m; m &= m - 1) j->closure[i0 + (size_t)__builtin_ctzll(m)]++;
        for (size_t t = 0; t < nt; t++) vis[touched[t]] = 0;
    }
    atomic_fetch_add(&j->visits, visits);
    free(vis);
    free(pend);
    free(touched);
    free(front);
    free(nextf);
    return NULL;
}

int kr_check(kr_checker *k, int nthreads, uint8_t *allowed, int *status, uint64_t *edge_visits,
             uint64_t *closure_size) {
    if (!k->finished) return KR_EREFUSED;
    job_t j = {.k = k, .allowed = allowed, .closure = closure_size};
    if (closure_size) memset(closure_size, 0, k->n * sizeof *closure_size);
    atomic_init(&j.next, 0);
    atomic_init(&j.visits, 0);
    memset(allowed, 0, k->n);
    if (nthreads < 1) nthreads = 1;
    pthread_t *t = calloc(nthreads, sizeof *t);
    for (int i = 0; i < nthreads; i++) pthread_create(&t[i], NULL, worker, &j);
    for (int i = 0; i < nthreads; i++) pthread_join(t[i], NULL);
    free(t);
    memcpy(status, k->status, k->n * sizeof(int));
    if (edge_visits) *edge_visits = atomic_load(&j.visits);
    return KR_OK;
}

void kr_stats(const kr_checker *k, uint64_t *nodes, uint64_t *edges) {
    if (nodes) *nodes = k->sets.n;
    if (edges) *edges = k->finished ? k->csr_off[k->sets.n] : k->ne;
}

void kr_free(kr_checker *k) {
    if (!k) return;
    for (size_t i = 0; i < k->nns; i++) free(k->ns_name[i]);
    free(k->ns_name);
    free(k->ns_id);
    intern_free(&k->sets);
    intern_free(&k->sids);
    free(k->root);
    free(k->tgt);
    free(k->status);
    free(k->is_target_set);
    free(k->edge);
    free(k->par);
    free(k->csr_off);
    free(k->csr_col);
    free(k->p_off);
    free(k->p_col);
    free(k);
}
