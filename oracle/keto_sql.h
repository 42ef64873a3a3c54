/*
 * keto_sql — BASELINE / TEST INFRASTRUCTURE ONLY (see keto_sql.c).
 * The reference's check over a real SQLite database through libsqlite3.so.0, one
 * read-only connection per worker thread.
 */
#ifndef KETO_SQL_H
#define KETO_SQL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KS_OK 0
#define KS_ENOTFOUND (-1)
#define KS_EINVAL (-2)
#define KS_ENOMEM (-3)
#define KS_SKIPPED (-9) /* not checked: the time budget ran out first */

typedef struct ks_db ks_db;
/* a new database file at path (replaced if present; removed by ks_db_free) */
ks_db *ks_db_create(const char *path, int page_size);
int ks_db_add_namespace(ks_db *d, int32_t id, const char *name);
/* rows as ketogpu_row_batch columns (include/ketogpu.h) */
int ks_db_add_rows_columnar(ks_db *d, size_t n, const int32_t *ns, const char *obj, const uint64_t *obj_off,
                            const char *rel, const uint64_t *rel_off, const uint8_t *kind, const char *sid,
                            const uint64_t *sid_off, const int32_t *ss_ns, const char *ss_obj,
                            const uint64_t *ss_obj_off, const char *ss_rel, const uint64_t *ss_rel_off,
                            const int64_t *commit_time);
/* commit and create the reference's indexes */
int ks_db_finish(ks_db *d);
void ks_db_free(ks_db *d);
/* SubjectIsAllowed for requests [0, n) on nthreads threads until `seconds` (0: no limit);
 * status[i] KS_OK / KS_EINVAL (nil subject) / KS_SKIPPED; *done requests answered,
 * *queries SQL statements issued */
int ks_check_batch(ks_db *d, size_t n, const char *const *ns, const char *const *obj, const char *const *rel,
                   const int *kind, const char *const *sid, const char *const *ss_ns, const char *const *ss_obj,
                   const char *const *ss_rel, int nthreads, double seconds, uint8_t *allowed, int *status,
                   size_t *done, long long *queries);

#ifdef __cplusplus
}
#endif
#endif
