/*
 * r2_check — TEST INFRASTRUCTURE ONLY (see r2_check.c): an independent checker of the R2
 * reachability formula over the raw row stream, for graphs the reference DFS restatement
 * (keto_oracle.c) cannot finish.  Shares no code with libketogpu.
 */
#ifndef R2_CHECK_H
#define R2_CHECK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KR_OK 0
#define KR_EREFUSED (-2) /* outside the checker's scope (wildcards, poisoned pages, nil) */
#define KR_ENOMEM (-3)

typedef struct kr_checker kr_checker;
kr_checker *kr_new(const int32_t *ns_ids, const char *const *ns_names, size_t nns);
/* the requests first (their targets select which subject-id rows are kept) */
int kr_add_requests(kr_checker *k, size_t n, const char *const *ns, const char *const *obj, const char *const *rel,
                    const int *kind, const char *const *sid, const char *const *ss_ns, const char *const *ss_obj,
                    const char *const *ss_rel);
/* rows as ketogpu_row_batch columns, grouped by (namespace_id, object, relation) */
int kr_add_rows_columnar(kr_checker *k, size_t n, const int32_t *ns, const char *obj, const uint64_t *obj_off,
                         const char *rel, const uint64_t *rel_off, const uint8_t *kind, const char *sid,
                         const uint64_t *sid_off, const int32_t *ss_ns, const char *ss_obj, const uint64_t *ss_obj_off,
                         const char *ss_rel, const uint64_t *ss_rel_off);
int kr_finish(kr_checker *k);
/* allowed[n] 0/1, status[n] KR_OK or KR_EREFUSED; *edge_visits: subject-set edges scanned */
/* closure_size: NULL, or per request the number of interior nodes its root reaches (|X(r)|) */
int kr_check(kr_checker *k, int nthreads, uint8_t *allowed, int *status, uint64_t *edge_visits,
             uint64_t *closure_size);
void kr_stats(const kr_checker *k, uint64_t *nodes, uint64_t *edges);
const char *kr_error(const kr_checker *k);
void kr_free(kr_checker *k);

#ifdef __cplusplus
}
#endif
#endif
