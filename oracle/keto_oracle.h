/*
 * keto_oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's (Ory Keto, Go) check and expand
 * algorithms over a raw relation-tuple table.  It exists to CHECK the MI355X
 * engine (libketogpu) and to time the reference algorithm on host cores
 * (bench.py `cpu_baseline`, kind "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never does.
 *
 * Reference semantics restated (all paths relative to the reference repo):
 *   GetRelationTuples       internal/persistence/sql/relationtuples.go:203-258
 *   toInternal              internal/persistence/sql/relationtuples.go:43-80
 *   pagination / tokens     internal/persistence/sql/persister.go:45-47,129-157
 *   namespace lookup        internal/driver/config/namespace_memory.go:29-47
 *   subjectIsAllowed        internal/check/engine.go:33-67
 *   checkOneIndirection...  internal/check/engine.go:69-91
 *   SubjectIsAllowed        internal/check/engine.go:93-95
 *   CheckAndAddVisited      internal/x/graph/graph_utils.go:13-35
 *   Subject.String/Equals   internal/relationtuple/definitions.go:164-170,253-267
 *   BuildTree               internal/expand/engine.go:30-98
 *   Tree JSON (node)        internal/expand/tree.go:85-91,156-162
 * Row order is the reference's ORDER BY (relationtuples.go:215) evaluated with
 * SQLite semantics (NULLs first, BINARY collation), the backend of the
 * reference's own tests; tests/test_oracle.py cross-checks it against sqlite3.
 *
 * Parity pinning: tests/golden/reference_cases.json (transcribed assertions of
 * the reference's own tests and docs expected outputs) — see DESIGN.md.
 */
#ifndef KETO_ORACLE_H
#define KETO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KO_OK 0
#define KO_ENOTFOUND (-1) /* herodot.ErrNotFound                      */
#define KO_EINVAL (-2)    /* malformed input / nil subject            */
#define KO_ENOMEM (-3)
#define KO_ETIMEOUT (-4)  /* ko_check_batch_budget: the request's time budget ran out */

#define KO_SUBJECT_ID 0
#define KO_SUBJECT_SET 1
#define KO_SUBJECT_NIL (-1)

typedef struct ko_store ko_store;

ko_store *ko_store_new(void);
void ko_store_free(ko_store *s);
/* namespaces in configuration order (lookups take the first match) */
int ko_add_namespace(ko_store *s, int32_t id, const char *name);
void ko_set_page_size(ko_store *s, int page_size);
/* row order of the backend: 0 SQLite (NULLs first, default), 1 Postgres (NULLs last) */
void ko_set_nulls_last(ko_store *s, int nulls_last);
/* one row of keto_relation_tuples; subject_id == NULL means a subject set */
int ko_add_row(ko_store *s, int32_t namespace_id, const char *object, const char *relation,
               const char *subject_id, int32_t ss_namespace_id, const char *ss_object,
               const char *ss_relation, int64_t commit_time);
/* columnar bulk append (same layout as ketogpu_row_batch, see include/ketogpu.h) */
int ko_add_rows_columnar(ko_store *s, size_t n, const int32_t *namespace_id,
                         const char *object_data, const uint64_t *object_off,
                         const char *relation_data, const uint64_t *relation_off,
                         const uint8_t *subject_kind, const char *subject_id_data,
                         const uint64_t *subject_id_off, const int32_t *ss_namespace_id,
                         const char *ss_object_data, const uint64_t *ss_object_off,
                         const char *ss_relation_data, const uint64_t *ss_relation_off,
                         const int64_t *commit_time);
/* sort rows by the ORDER BY clause; presorted=1 only verifies (returns KO_EINVAL if not sorted) */
int ko_finalize(ko_store *s, int presorted);
size_t ko_num_rows(const ko_store *s);

/* SubjectIsAllowed; *allowed = 0/1.  Returns KO_OK or a negative error. */
int ko_check(const ko_store *s, const char *ns, const char *obj, const char *rel, int subject_kind,
             const char *subject_id, const char *ss_ns, const char *ss_obj, const char *ss_rel,
             int *allowed);

/* many checks on nthreads threads; status[i] = KO_OK or error, allowed[i] = 0/1 */
int ko_check_batch(const ko_store *s, size_t n, const char *const *ns, const char *const *obj,
                   const char *const *rel, const int *subject_kind, const char *const *subject_id,
                   const char *const *ss_ns, const char *const *ss_obj, const char *const *ss_rel,
                   int nthreads, uint8_t *allowed, int *status);

/* ko_check_batch with a time budget per request (the full-size pins: a negative check of
 * a power-law graph walks ~10^6 groups); status KO_ETIMEOUT for the requests that ran out */
int ko_check_batch_budget(const ko_store *s, size_t n, const char *const *ns, const char *const *obj,
                          const char *const *rel, const int *subject_kind, const char *const *subject_id,
                          const char *const *ss_ns, const char *const *ss_obj, const char *const *ss_rel,
                          int nthreads, double seconds_per_request, uint8_t *allowed, int *status);

/* BuildTree; *json receives the tree as the reference's JSON (or "null"); free with ko_free */
int ko_expand(const ko_store *s, int subject_kind, const char *subject_id, const char *ss_ns,
              const char *ss_obj, const char *ss_rel, int rest_depth, char **json);

/* GetRelationTuples page as JSON list of {namespace,object,relation,subject_*}; for tests */
int ko_get_page(const ko_store *s, const char *ns, const char *obj, const char *rel, int page,
                char **json, int *has_next);

void ko_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
