/*
 * ketogpu.h — C ABI of the MI355X batched permission-check engine (libketogpu.so).
 *
 * This is the drop-in boundary for Ory Keto's evaluation engines.  Every entry
 * point below replaces a reference interface (paths relative to the reference
 * repository); the Go side binds it through cgo.
 *
 *   ketogpu_builder_*      new persistence-side snapshot loader; replaces the
 *                          per-node SQL reads of (*Persister).GetRelationTuples
 *                          internal/persistence/sql/relationtuples.go:203-258
 *   ketogpu_check          (*check.Engine).SubjectIsAllowed
 *                          internal/check/engine.go:93-95 (recursion :33-91)
 *   ketogpu_resolve /      the same, split into host resolution (strings -> node
 *   ketogpu_check_ids /    ids) and a batched device traversal over ids with
 *   ketogpu_queries_*      inputs resident in HBM
 *   ketogpu_expand         (*expand.Engine).BuildTree internal/expand/engine.go:30-98
 *   ketogpu_tree_*         expand.Tree / its JSON codec internal/expand/tree.go:26-30,85-91,156-162
 *
 * Conventions: plain C types only; all input memory is copied (cgo pointer rules);
 * opaque handles are owned by the library; result buffers are caller-allocated.
 * Functions return KETOGPU_OK or a positive KETOGPU_E* code; ketogpu_last_error()
 * returns a thread-local message for the last failure on the calling thread.
 * Error mapping (herodot): ENOTFOUND -> ErrNotFound (404), EINVAL -> ErrBadRequest
 * (400), EDEVICE/ENOMEM -> ErrInternalServerError (500).
 */
#ifndef KETOGPU_H
#define KETOGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KETOGPU_ABI_VERSION 9 /* 9: plan label in the two-tier mode (tier stats label_*);
                                 8: 2-hop reachability labels (plan label), run stats
                                    label_* / rest_*;
                                 7: two-tier partitioned mode (ketogpu_core_*, ketogpu_tier_*);
                                 6: partitioned rounds behind the C ABI (comm, part_engine);
                                 5: writable snapshots (in-place writes, engine sync);
                                 4: ketogpu_shard_*, part_new over a shard; 3: host_alloc, multi */

#define KETOGPU_OK 0
#define KETOGPU_ENOTFOUND 1 /* unknown namespace (herodot.ErrNotFound)              */
#define KETOGPU_EINVAL 2    /* malformed input, nil subject, unsorted rows          */
#define KETOGPU_EDEVICE 3   /* HIP runtime / device failure                          */
#define KETOGPU_ENOMEM 4    /* host or device allocation failure                    */
#define KETOGPU_ECOLLISION 5 /* partitioned loader: 64-bit node hash collision; reload
                                with another ketogpu_shard_opts.salt                 */

#define KETOGPU_SUBJECT_ID 0
#define KETOGPU_SUBJECT_SET 1
#define KETOGPU_SUBJECT_NIL (-1)

#define KETOGPU_NODE_NONE 0xFFFFFFFFu /* no such node / root with no tuples      */
#define KETOGPU_NODE_NOT_OWNED 0xFFFFFFFEu /* ketogpu_shard_resolve_batch: another rank
                                              owns this node and resolves it          */

/* builder flags */
#define KETOGPU_BUILD_SORT 1u /* rows are NOT in ORDER BY order: sort them with the
                                  snapshot's row order (below) */
/* Row order of the backend the rows come from.  The ORDER BY of
 * relationtuples.go:215 is executed by the backend, and only NULL placement and string
 * collation differ between backends: SQLite (tests, default), MySQL with a binary
 * collation and CockroachDB put NULLs first; Postgres puts NULLs last — so a Postgres
 * group lists its subject-id rows (subject_id NOT NULL) before its subject-set rows.
 * Strings compare bytewise in both orders (SQLite BINARY, MySQL *_bin, Postgres "C"
 * collation, CockroachDB).  Locale collations are not modelled (expand order under them is
 * unpinned).  The order only matters where the library itself places rows: sorting
 * (KETOGPU_BUILD_SORT) and ketogpu_snapshot_apply; rows appended in order are kept. */
#define KETOGPU_ORDER_NULLS_LAST 2u /* Postgres ORDER BY (NULLS LAST, C collation) */
/* Writable snapshot (ketogpu_snapshot_write): the device rows are laid out with free slots
 * (2 + 1/8 of each row part) and ids are reserved for new subjects,
 * so a write batch patches the rows it touches in place instead of rebuilding the graph. */
#define KETOGPU_BUILD_WRITABLE 4u

typedef struct ketogpu_builder ketogpu_builder;
typedef struct ketogpu_snapshot ketogpu_snapshot;
typedef struct ketogpu_engine ketogpu_engine;
typedef struct ketogpu_queries ketogpu_queries;
typedef struct ketogpu_tree ketogpu_tree;

/* namespace.Namespace{ID, Name} (internal/namespace/definitons.go:8-12), config order */
typedef struct {
    int32_t id;
    const char *name;
} ketogpu_namespace;

/* A batch of keto_relation_tuples rows, columnar (one row per index; string column c of
 * row i is c_data[c_off[i] .. c_off[i+1]), offsets have n+1 entries).  Row layout follows
 * RelationTuple (internal/persistence/sql/relationtuples.go:18-31): subject_kind 0 =
 * subject_id row (ss_* ignored), 1 = subject-set row (subject_id ignored).
 * Rows of one snapshot must arrive in the backend's
 *   ORDER BY nid, namespace_id, object, relation, subject_id, subject_set_namespace_id,
 *            subject_set_object, subject_set_relation, commit_time   (relationtuples.go:215)
 * order across all append calls, for ONE nid (persister.go:117-119), unless the builder
 * was created with KETOGPU_BUILD_SORT. */
typedef struct {
    size_t n;
    const int32_t *namespace_id;
    const char *object_data;
    const uint64_t *object_off;
    const char *relation_data;
    const uint64_t *relation_off;
    const uint8_t *subject_kind;
    const char *subject_id_data;
    const uint64_t *subject_id_off;
    const int32_t *ss_namespace_id;
    const char *ss_object_data;
    const uint64_t *ss_object_off;
    const char *ss_relation_data;
    const uint64_t *ss_relation_off;
} ketogpu_row_batch;

typedef struct {
    int32_t page_size; /* GetRelationTuples page size; 0 -> 100 (persister.go:68-70) */
    uint32_t flags;    /* KETOGPU_BUILD_* */
} ketogpu_build_opts;

typedef struct {
    uint64_t num_rows;           /* rows appended                                  */
    uint64_t num_bad_rows;       /* rows whose namespace ids are not configured    */
    uint64_t num_groups;         /* distinct (namespace_id, object, relation)      */
    uint64_t num_nodes;          /* N: subject nodes (subject ids + subject sets)  */
    uint64_t num_expandable;     /* Nx: nodes whose query returns >= 1 row         */
    uint64_t num_interior;       /* Ni: expandable nodes that are also subjects    */
    uint64_t num_edges;          /* rows kept after page-poison truncation         */
    uint64_t num_interior_edges; /* deduplicated edges into interior nodes         */
    uint64_t num_rev_edges;      /* deduplicated reverse edges                     */
    uint64_t num_wildcard_nodes; /* subject sets with an empty field (R5)           */
    uint64_t num_ambiguous_nodes;/* nodes sharing a Subject.String() key (R4)      */
    double build_seconds;
} ketogpu_snapshot_stats;

/* ----------------------------------------------------------------- snapshot */
int ketogpu_builder_new(const ketogpu_namespace *namespaces, size_t num_namespaces,
                        const ketogpu_build_opts *opts, ketogpu_builder **out);
int ketogpu_builder_append(ketogpu_builder *b, const ketogpu_row_batch *rows);
/* consumes b (also on failure) */
int ketogpu_builder_finish(ketogpu_builder *b, ketogpu_snapshot **out);
void ketogpu_builder_free(ketogpu_builder *b);
void ketogpu_snapshot_free(ketogpu_snapshot *s);
int ketogpu_snapshot_stats_get(const ketogpu_snapshot *s, ketogpu_snapshot_stats *out);

/* Write-path freshness (R14): the next snapshot version = the base's
 * rows with one TransactRelationTuples batch applied (internal/persistence/sql/
 * relationtuples.go:271-278): inserts join their group after equal rows (commit_time
 * order), then every row matching a delete is removed (:178-201).  Row order follows
 * the base snapshot's row order (KETOGPU_ORDER_*).  The base stays valid; engines built on
 * the new version answer with the write applied.  inserts/deletes may be NULL. */
int ketogpu_snapshot_apply(const ketogpu_snapshot *base, const ketogpu_row_batch *inserts,
                           const ketogpu_row_batch *deletes, ketogpu_snapshot **out);

/* Namespace-configuration reload (internal/driver/config/provider.go:87-110: Keto drops
 * its namespace manager whenever KeyNamespaces changes): the next version holds the base's
 * rows under the new configuration, so page poisoning (R7) and name resolution follow it —
 * rows of a namespace id that is no longer configured poison their pages, rows of a
 * re-added one are visible again.  Duplicate names or ids are refused (KETOGPU_EINVAL). */
int ketogpu_snapshot_set_namespaces(const ketogpu_snapshot *base, const ketogpu_namespace *namespaces,
                                    size_t num_namespaces, ketogpu_snapshot **out);

/* In-place write (R14 at O(delta)) on a KETOGPU_BUILD_WRITABLE
 * snapshot: the same TransactRelationTuples semantics as ketogpu_snapshot_apply (inserts
 * after equal rows, then every row matching a delete removed), applied to THIS snapshot:
 * the touched groups' rows (host: expand, exact checks, resolution) and the touched device
 * rows (a patch list each engine uploads at its next call, or at ketogpu_engine_sync).
 * Cost: O(rows of the touched groups + touched device rows), independent of the graph.
 * A batch the free slots cannot represent leaves the snapshot unchanged and reports
 * applied = 0 with a reason; the caller then builds the next version with
 * ketogpu_snapshot_apply (which keeps the snapshot writable).  Not representable: a row
 * that creates a group or makes an expandable node interior (node classes are fixed
 * between rebuilds), rows with unconfigured namespace ids or touching a poisoned group (R7),
 * snapshots with wildcard subject sets (R5) or shared Subject.String() keys (R4), a new
 * subject whose key is shared, a full row, no reserved ids left.  Concurrent calls on the
 * snapshot and its engines are serialized against the write (reader/writer lock).
 * Nodes keep their class after their last row is deleted (an expandable node without rows
 * answers like a non-expandable one). */
#define KETOGPU_WRITE_APPLIED 0
#define KETOGPU_WRITE_NOT_WRITABLE 1
#define KETOGPU_WRITE_WILDCARD 2   /* R5 wildcard subject sets in the snapshot or the batch */
#define KETOGPU_WRITE_POISON 3     /* unconfigured namespace id, or a poisoned group (R7) */
#define KETOGPU_WRITE_CLASS 4      /* a new group, or an expandable node becoming interior */
#define KETOGPU_WRITE_AMBIGUOUS 5  /* shared Subject.String() keys (R4) */
#define KETOGPU_WRITE_FULL 6       /* a touched row has no free slot left */
#define KETOGPU_WRITE_RESERVE 7    /* no reserved node id left for a new subject */
#define KETOGPU_WRITE_FANOUT 8     /* a record count change would re-upload more rows than
                                      KETOGPU_WRITE_FANOUT_MAX (env, default 65536) */
typedef struct {
    int32_t applied;          /* 1: written in place; 0: unchanged, see reason */
    int32_t reason;           /* KETOGPU_WRITE_* */
    uint64_t rows_inserted;   /* rows added to groups */
    uint64_t rows_deleted;    /* rows removed (all duplicates of a deleted tuple) */
    uint64_t groups_touched;
    uint64_t device_rows;     /* device rows patched (forward + reverse) */
    uint64_t new_nodes;       /* subjects that got a reserved id */
    uint64_t version;         /* the snapshot's write version after the call */
    double seconds;           /* host time of the call */
} ketogpu_write_result;
int ketogpu_snapshot_write(ketogpu_snapshot *s, const ketogpu_row_batch *inserts, const ketogpu_row_batch *deletes,
                           ketogpu_write_result *result);
uint64_t ketogpu_snapshot_version(const ketogpu_snapshot *s);

/* Persisted snapshots (fast restart): a versioned binary image of
 * a finished snapshot.  Loading rebuilds only the derived indexes; a file written by a
 * different format version is refused with KETOGPU_EINVAL. */
int ketogpu_snapshot_save(const ketogpu_snapshot *s, const char *path);
int ketogpu_snapshot_load(const char *path, ketogpu_snapshot **out);

/* Read-only view of the device graph as built on the host (for tools and tests; the
 * pointers live as long as the snapshot).  Node ids: [0, num_interior) interior,
 * [num_interior, num_expandable) other expandable nodes, the rest never expand. */
typedef struct {
    uint32_t num_nodes, num_expandable, num_interior;
    const uint64_t *fint_off; /* num_expandable + 1 */
    const uint32_t *fint_col; /* interior successors of each expandable node */
    const uint64_t *rev_off;  /* num_nodes + 1 */
    const uint32_t *rev_col;  /* expandable predecessors of each node */
} ketogpu_graph_view;
int ketogpu_snapshot_graph(const ketogpu_snapshot *s, ketogpu_graph_view *out);

/* Plan "core"'s record arrays (keto_amd/csrc/core_index.hpp), built on the host the way an
 * engine builds them, for tools and tests (the engine builds its own; KETOGPU_UNITS=core).
 * Per direction (0 forward, 1 backward) one array of 16-byte records {node, deg, begin,
 * pad}: core rows (the rows among interior nodes), closure rows (pad bit 31: TERMINAL
 * entries), node blocks of the seed rows (fint(v) / rev(v); the head record of node v's
 * block {count, first record low, high, 0}) and overflow rows.  A record's deg/begin name
 * the node's expansion row in the same array; pad bit 30 = that row is a closure row.
 * closure_cap[d] = 0: no closure rows; block[d] = 0: block size chosen from the rows. */
typedef struct ketogpu_core_index ketogpu_core_index;
typedef struct {
    const uint32_t *records; /* 4 x u32 per record */
    uint64_t num_records;
    uint64_t block_base;     /* record index of node 0's block */
    uint32_t block_records;  /* records per node block: 4, 8, 16 or 32 */
    uint64_t overflow_rows;  /* seed rows kept outside their block */
    uint64_t closure_nodes, closure_entries;
} ketogpu_core_records;
int ketogpu_core_index_build(const ketogpu_snapshot *s, const uint32_t closure_cap[2], const uint32_t block[2],
                             ketogpu_core_index **out);
int ketogpu_core_index_view(const ketogpu_core_index *c, int direction, ketogpu_core_records *out);
void ketogpu_core_index_free(ketogpu_core_index *c);

/* Plan "label"'s 2-hop reachability labels (keto_amd/csrc/labels.hpp) as an engine builds
 * them, for tools and tests.  Interior nodes are ranked; Lin(v) / Lout(v) hold the ranks of
 * the landmarks that reach v / that v reaches (the first 64 landmarks as a bit mask), so
 * that a ->* b <=> Lout(a) meets Lin(b).  Per request:
 *   S(t) = Lin(v) for every interior v in rev(t), plus rev(t)'s other entries (node ids);
 *   P(r) = Lout(r) (r interior), else {r} + Lout(c) for every c in fint(r);
 *   allowed(r, t) <=> S(t) and P(r) share an entry or their masks share a bit.
 * One head per node (S: every node, P: every expandable node) of s_head_words /
 * p_head_words u32 (8, 16 or 32; 0 = chosen from the list lengths):
 *   [count, overflow start / 16, mask lo, mask hi, entries ascending, 0xFFFFFFFF pad];
 * a list longer than head - 4 entries lies whole at words 16 x (overflow start). */
typedef struct ketogpu_label_index ketogpu_label_index;
typedef struct {
    uint32_t s_head_words, p_head_words;
    const uint32_t *s_words, *p_words;
    uint64_t num_s_words, num_p_words;
    uint64_t s_nodes, p_nodes;
    uint64_t s_entries, p_entries;   /* list entries (masks not counted) */
    uint64_t s_overflow, p_overflow; /* lists kept outside their head */
    uint64_t label_entries;          /* Lin + Lout entries */
    double pll_ms, build_ms;         /* the labels / labels and heads (host) */
} ketogpu_label_view;
int ketogpu_label_index_build(const ketogpu_snapshot *s, uint32_t s_head_words, uint32_t p_head_words,
                              ketogpu_label_index **out);
int ketogpu_label_index_view(const ketogpu_label_index *l, ketogpu_label_view *out);
void ketogpu_label_index_free(ketogpu_label_index *l);

/* ------------------------------------------------------------------- check */
/* relationtuple.Subject: SubjectID{ID} or SubjectSet{Namespace, Object, Relation}
 * (internal/relationtuple/definitions.go:39-41,103-118) */
typedef struct {
    int32_t kind; /* KETOGPU_SUBJECT_* */
    const char *id;
    const char *ns;
    const char *obj;
    const char *rel;
} ketogpu_subject;

/* InternalRelationTuple used as a check request (definitions.go:95-100); an empty
 * namespace/object/relation is "no filter", as in GetRelationTuples. */
typedef struct {
    const char *ns;
    const char *obj;
    const char *rel;
    ketogpu_subject subject;
} ketogpu_check_request;

/* Host resolution of one request to node ids.  *root is an expandable node or
 * KETOGPU_NODE_NONE (the query returns no tuples, or its namespace is unknown: false);
 * *target is a node or KETOGPU_NODE_NONE (the subject appears in no tuple: false).
 * Returns KETOGPU_EINVAL for a nil subject; returns KETOGPU_ENOTFOUND with *root =
 * KETOGPU_NODE_NONE when the root is a wildcard query that matches no snapshot node
 * (use ketogpu_check for those). */
int ketogpu_resolve(const ketogpu_snapshot *s, const ketogpu_check_request *req, uint32_t *root,
                    uint32_t *target);

/* A batch of check requests, columnar like ketogpu_row_batch (string column c of request
 * i is c_data[c_off[i] .. c_off[i+1])).  subject_kind: 0 subject id (sid columns), 1
 * subject set (ss_* columns), 255 nil subject; NULL means all subject ids. */
typedef struct {
    size_t n;
    const char *ns_data;
    const uint64_t *ns_off;
    const char *obj_data;
    const uint64_t *obj_off;
    const char *rel_data;
    const uint64_t *rel_off;
    const uint8_t *subject_kind;
    const char *sid_data;
    const uint64_t *sid_off;
    const char *ss_ns_data;
    const uint64_t *ss_ns_off;
    const char *ss_obj_data;
    const uint64_t *ss_obj_off;
    const char *ss_rel_data;
    const uint64_t *ss_rel_off;
} ketogpu_request_batch;

/* ketogpu_resolve for a whole batch; status[i] as ketogpu_resolve's return value
 * (KETOGPU_OK, KETOGPU_EINVAL for nil subjects, KETOGPU_ENOTFOUND for wildcard roots
 * without a node).  status may be NULL. */
int ketogpu_resolve_batch(const ketogpu_snapshot *s, const ketogpu_request_batch *reqs, uint32_t *roots,
                          uint32_t *targets, int32_t *status);

typedef struct {
    int32_t device;             /* HIP device ordinal                                */
    uint32_t max_words_per_round; /* 64-check words traversed together; 0 = auto      */
    uint64_t state_budget_bytes;  /* HBM for traversal state; 0 = auto (<= 1/3 free)  */
} ketogpu_engine_opts;

/* uploads the snapshot's device graph (forward interior CSR + reverse CSR) to HBM */
int ketogpu_engine_new(const ketogpu_snapshot *s, const ketogpu_engine_opts *opts,
                       ketogpu_engine **out);
void ketogpu_engine_free(ketogpu_engine *e);

/* SubjectIsAllowed for n requests: allowed[i] in {0,1}; status[i] = KETOGPU_OK or
 * KETOGPU_EINVAL (nil subject).  Unknown namespaces yield allowed = 0 (engine.go:75-77).
 * The function itself fails only on device/alloc errors. */
int ketogpu_check(ketogpu_engine *e, const ketogpu_check_request *reqs, size_t n, uint8_t *allowed,
                  int32_t *status);

/* id-level batch: roots/targets from ketogpu_resolve; allowed_bits / flagged_bits have
 * ceil(n/64) words, bit i%64 of word i/64 for request i.  A flagged request touched a
 * node whose Subject.String() key is shared with another node (R4 in DESIGN.md): its bit
 * is only exact after re-evaluation with the sequential semantics (ketogpu_check does
 * that itself).  flagged_bits may be NULL.  Host to host: the requests are copied to HBM
 * in chunks that overlap the traversal of the chunks before them, ids are validated on
 * the device (an id outside the snapshot fails the call with KETOGPU_EINVAL), and the
 * result bits come back with the run's one host synchronization.  This is the batch
 * call SURVEY.md 8(d) times. */
int ketogpu_check_ids(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                      uint64_t *allowed_bits, uint64_t *flagged_bits);

/* Pinned host memory (hipHostMalloc) for request and result arrays.  A batch whose
 * roots/targets live here is copied by DMA at full PCIe rate; the cgo micro-batcher
 *  fills such a buffer in place instead of a Go slice, which it has to
 * copy into C memory anyway (cgo pointer rules).  Any host memory works with
 * ketogpu_check_ids; pageable memory is staged by the HIP runtime. */
int ketogpu_host_alloc(size_t bytes, void **out);
void ketogpu_host_free(void *p);

/* ------------------------------------------------------ replicated multi-GPU */
/* One engine per listed device over the same snapshot (the graph replicated in every
 * GPU's HBM, SURVEY.md 8(e) "Replicated"); replaces scaling out by more Keto processes
 * (internal/driver/daemon.go:87-159) with one PermissionEngine per process
 * (internal/driver/registry_default.go:158-163) that drives the whole node.
 * ketogpu_multi_check_ids splits the batch into ketogpu_multi_size() contiguous ranges of
 * whole 64-request words (ketogpu_multi_range), runs ketogpu_check_ids on every device
 * concurrently from one host thread per device and writes each range's bits at its
 * offset of allowed_bits / flagged_bits.  No communication between devices. */
typedef struct ketogpu_multi ketogpu_multi;
int ketogpu_multi_new(const ketogpu_snapshot *s, const int32_t *devices, size_t num_devices,
                      const ketogpu_engine_opts *opts, ketogpu_multi **out);
void ketogpu_multi_free(ketogpu_multi *m);
size_t ketogpu_multi_size(const ketogpu_multi *m);
/* the engine of device slot i (statistics); owned by m */
ketogpu_engine *ketogpu_multi_engine(ketogpu_multi *m, size_t i);
int ketogpu_multi_check_ids(ketogpu_multi *m, const uint32_t *roots, const uint32_t *targets, size_t n,
                            uint64_t *allowed_bits, uint64_t *flagged_bits);
/* requests [*begin, *end) of part i when n requests are split into `parts` ranges */
void ketogpu_multi_range(size_t n, size_t parts, size_t i, size_t *begin, size_t *end);

/* device-resident query sets: upload once, run many times (results stay in HBM) */
int ketogpu_queries_upload(ketogpu_engine *e, const uint32_t *roots, const uint32_t *targets,
                           size_t n, ketogpu_queries **out);
int ketogpu_queries_run(ketogpu_engine *e, ketogpu_queries *q);
int ketogpu_queries_download(ketogpu_engine *e, const ketogpu_queries *q, uint64_t *allowed_bits,
                             uint64_t *flagged_bits);
/* the same call as ketogpu_queries_run, enqueued on the engine's stream without waiting for
 * the device when the engine can prove that no request of the batch needs the second stage
 * (plan label, no head marked unlabelled, no wildcard root): batches are then pipelined, the
 * way a server enqueues batch k+1 while batch k runs (Keto's check handler answers each
 * request when its batch's bits are back: internal/check/handler.go).  *queued = 1 when the
 * call returned before the device finished — its results are complete once
 * ketogpu_queries_download or ketogpu_engine_wait returns, and a device error of the call is
 * reported by that later call; 0: it ran as ketogpu_queries_run.  (queued may be NULL.) */
int ketogpu_queries_run_async(ketogpu_engine *e, ketogpu_queries *q, int *queued);
/* waits for every call enqueued on the engine (ketogpu_queries_run_async) */
int ketogpu_engine_wait(ketogpu_engine *e);
void ketogpu_queries_free(ketogpu_queries *q);

/* statistics of the last run on this engine (for the roofline report) */
typedef struct {
    uint64_t checks;
    uint64_t rounds;
    uint64_t levels;            /* BFS levels summed over rounds                  */
    uint64_t frontier_entries;  /* (word, node) entries expanded                  */
    uint64_t interior_edges;    /* interior edges scanned by the push kernel      */
    uint64_t rev_edges;         /* reverse edges scanned by the pull kernel       */
    uint64_t touched;           /* (word, node) visited entries reset             */
    uint64_t bytes_push;        /* algorithmic bytes of the push (expand) kernel  */
    uint64_t bytes_pull;        /* algorithmic bytes of the pull kernel           */
    uint64_t bytes_total;       /* algorithmic bytes of all kernels               */
    double ms_push;             /* summed device time of push launches (hipEvent) */
    double ms_pull;
    double ms_total;            /* device time, first to last kernel              */
    uint64_t push_launches;
    uint64_t overflow_retries;
    /* LDS unit path (one launch: whole BFS + pull per 16-request unit in LDS) */
    uint64_t spilled_units;     /* units that spilled out of an LDS table (all passes) */
    uint64_t unit_rows;         /* rows opened (forward offsets + reverse offsets) */
    uint64_t unit_edges;        /* interior edges scanned                         */
    uint64_t unit_rev;          /* reverse entries scanned                        */
    uint64_t bytes_unit;        /* algorithmic HBM bytes of the unit kernel       */
    double ms_unit;             /* device time of the unit kernels (hipEvent)     */
    uint64_t spilled_requests;  /* single requests run on the global path         */
    uint64_t unit_launches;     /* unit-kernel launches (cascade passes)          */
    uint64_t main_bytes;        /* algorithmic HBM bytes of the first unit pass   */
    double main_ms;             /* its device time (hipEvent)                     */
    int32_t plan;               /* first stage of the run: 0 global path only, 1 bidi,
                                 * 2 forward unit2 (v2), 3 one-wave units, 4 unit v1,
                                 * 5 lite, 6 core (lite with closure rows), 7 label.
                                 * KETOGPU_UNITS=auto (default) tries bidi (128- and 64-
                                 * entry pending lists), v2 and (with hubs) the global path
                                 * alone on the first two batches of
                                 * >= 65536 requests, then keeps the fastest; those two
                                 * calls run every candidate (same results)              */
    uint32_t plan_lists;        /* bidi: pending-list entries of the first stage        */
    uint32_t hubs;              /* hub index: hubs (0 = off); searches stop at hubs and
                                 * read their precomputed closures (power-law graphs)   */
    uint32_t hub_words;         /* 64-bit words per interior node of the hub closures   */
    double hub_build_ms;        /* one-time hub closure build at engine creation        */
    uint32_t plan_unit;         /* bidi: requests per first-stage unit (16 or 8)        */
    /* plan 6 "core" (lite over its own record arrays with CLOSURE rows: an interior node
     * whose forward / backward closure has at most cap nodes expands into all of it in one
     * level; KETOGPU_CLOSURE="cap_f,cap_b") */
    uint32_t closure_cap_f, closure_cap_b;  /* 0, 0 when the plan is off                */
    uint64_t closure_nodes_f, closure_nodes_b;      /* nodes with a closure row          */
    uint64_t closure_entries_f, closure_entries_b;  /* records in closure rows           */
    double core_build_ms;       /* one-time build of the core arrays at engine creation */
    /* plan 7 "label" (2-hop reachability labels, labels.hpp: one intersection of two short
     * sorted lists per request; requests without labels — wildcard roots — go to a second
     * stage, plan lite over the listed requests) */
    int32_t label_on;           /* 1: labels built                                      */
    double label_coverage;      /* share of the non-empty S heads with a label (1 unless
                                 * KETOGPU_LABEL_REST_PERMILLE marks some for the second stage) */
    double label_build_ms;      /* one-time build at engine creation (labels + heads)   */
    uint32_t label_s_head;      /* S / P head words (8, 16 or 32)                       */
    uint32_t label_p_head;
    double label_pll_ms;        /* of which the 2-hop labels                            */
    uint64_t label_bytes;       /* S + P arrays in HBM                                  */
    uint64_t label_entries;     /* Lin + Lout entries                                   */
    uint64_t rest_requests;     /* requests of this run answered by the second stage    */
    uint64_t full_requests;     /* requests whose overflowing list the dense pass searched */
    double rest_ms;             /* second stage + statistics (events between kernels)   */
    /* plan label on a writable snapshot (label_update: heads rewritten in place per write) */
    uint64_t label_rewritten;   /* heads rewritten after writes                          */
    uint64_t label_marked;      /* heads marked "no label" (second stage) since the build */
    uint64_t label_relabels;    /* rebuilds from the current rows                        */
} ketogpu_run_stats;
int ketogpu_engine_last_stats(const ketogpu_engine *e, ketogpu_run_stats *out);
/* every_kernel = 1: host-to-host batches (ketogpu_check_ids from pinned memory), and plan
 * label's device-resident batches, record a timing event between the call's kernels, so
 * last_stats' main_ms is the first stage's own device time (each event pair costs a few
 * microseconds of idle GPU between the launches); 0 (default): one event pair around the
 * whole call (KETOGPU_EVENTS=all sets 1 at creation) */
int ketogpu_engine_set_events(ketogpu_engine *e, int every_kernel);

/* Upload the device rows patched by ketogpu_snapshot_write since the engine's last sync
 * (every check entry point also does this first).  ms: host time of the sync (may be NULL);
 * rows: device rows uploaded (may be NULL). */
int ketogpu_engine_sync(ketogpu_engine *e, double *ms, uint64_t *rows);
/* Test hook: the engine's device rows and edge records compared entry by entry with the
 * snapshot's host rows (after a sync); mismatches = entries that differ. */
int ketogpu_engine_check_graph(ketogpu_engine *e, uint64_t *mismatches);
/* Test hook: plan label's S (side 0) or P (side 1) head array as the engine built it on the
 * device (the layout of ketogpu_label_view); *words = its length in u32 words (0: no
 * labels), *head_words its head size; copied into out when capacity >= *words. */
int ketogpu_engine_label_heads(ketogpu_engine *e, int side, uint32_t *out, uint64_t capacity, uint64_t *words,
                               uint32_t *head_words);

/* ----------------------------------------------- partition-aware loader */
/* BASELINE config #5 (SURVEY.md 8(e) "Partitioned"): a graph that fits neither one GPU nor
 * one host.  Every rank streams the same ordered row read the single-GPU loader takes
 * (ketogpu_builder_*; internal/persistence/sql/relationtuples.go:203-258 with the ORDER
 * BY of :215, one nid, persister.go:94-96) and keeps only what it owns: node v (a typed
 * subject, internal/relationtuple/definitions.go:253-267) belongs to rank
 * hash(v, salt) % world; a rank keeps the rows of the groups it owns (forward rows) and
 * the rows whose subject it owns (reverse rows), after the reference's page poisoning
 * (R7), so no rank interns or holds the whole graph.  Owners number their nodes; the ids
 * of referenced nodes owned elsewhere come from one exchange the caller carries out
 * (keto_amd/partition.py: torch.distributed all_to_all / all_gather):
 *   builder_new/append.../finish -> counts -> [all_gather] -> set_layout
 *   -> queries -> [all_to_all] -> answer -> [all_to_all] -> apply
 *   -> claims -> [all_to_all] -> check_claims -> [all_reduce: any ambiguous key -> refuse]
 * Graphs the partitioned engine does not evaluate are refused on every rank alike:
 * wildcard subject sets (R5) and rows out of ORDER BY order with KETOGPU_EINVAL, shared
 * Subject.String() keys (R4) by check_claims' count.  Node ids: within each class (interior,
 * other expandable, never expanded) ids interleave the ranks, so owner and local index are
 * arithmetic (partition.hip); interior ids stay the smallest. */
typedef struct ketogpu_shard_builder ketogpu_shard_builder;
typedef struct ketogpu_shard ketogpu_shard;
typedef struct {
    int32_t page_size; /* GetRelationTuples page size; 0 -> 100                        */
    uint32_t flags;    /* KETOGPU_ORDER_* (rows must arrive in ORDER BY order)          */
    int32_t rank, world; /* world <= 64                                                 */
    uint64_t salt;     /* node hash salt; retry another after KETOGPU_ECOLLISION       */
} ketogpu_shard_opts;
typedef struct {
    uint64_t rows, bad_rows;             /* rows streamed; rows with unknown namespaces */
    uint64_t owned_nodes, owned_interior, owned_expandable;
    uint64_t forward_edges;              /* kept forward row entries (before dedup)     */
    uint64_t interior_forward_edges;     /* device forward rows (interior, deduplicated) */
    uint64_t reverse_edges;              /* reverse row entries                         */
    uint64_t queries;                    /* distinct referenced nodes (id exchange)     */
    uint64_t ambiguous_keys;             /* check_claims: shared String() keys found    */
    uint64_t num_interior, num_expandable, num_nodes; /* global id layout (Ni, Nx, N)   */
    uint64_t host_bytes;                 /* peak bytes of the loader's own arrays       */
    double seconds;                      /* streaming time                              */
} ketogpu_shard_stats;
int ketogpu_shard_builder_new(const ketogpu_namespace *namespaces, size_t num_namespaces,
                              const ketogpu_shard_opts *opts, ketogpu_shard_builder **out);
int ketogpu_shard_builder_append(ketogpu_shard_builder *b, const ketogpu_row_batch *rows);
/* consumes b (also on failure) */
int ketogpu_shard_builder_finish(ketogpu_shard_builder *b, ketogpu_shard **out);
void ketogpu_shard_builder_free(ketogpu_shard_builder *b);
void ketogpu_shard_free(ketogpu_shard *s);
/* this rank's node counts per class; every rank's (world x 3, rank order) to set_layout */
int ketogpu_shard_counts(const ketogpu_shard *s, uint64_t counts[3]);
int ketogpu_shard_set_layout(ketogpu_shard *s, const uint64_t *all_counts);
/* distinct node hashes this rank references, grouped by owner (counts[world]) */
uint64_t ketogpu_shard_query_count(const ketogpu_shard *s);
int ketogpu_shard_queries(const ketogpu_shard *s, uint64_t *hashes, uint64_t capacity, uint64_t *counts);
/* owner side: the global ids of received hashes (all owned by this rank) */
int ketogpu_shard_answer(const ketogpu_shard *s, const uint64_t *hashes, uint64_t n, uint32_t *ids);
/* the answers, in the order of ketogpu_shard_queries: builds the device rows */
int ketogpu_shard_apply(ketogpu_shard *s, const uint32_t *ids, uint64_t n);
/* R4: (String() key hash, node hash) pairs of owned nodes whose key another node could
 * share, grouped by the key hash's owner; the receiver counts keys held by >= 2 nodes */
uint64_t ketogpu_shard_claim_count(const ketogpu_shard *s);
int ketogpu_shard_claims(const ketogpu_shard *s, uint64_t *pairs, uint64_t capacity, uint64_t *counts);
int ketogpu_shard_check_claims(ketogpu_shard *s, const uint64_t *pairs, uint64_t n, uint64_t *ambiguous);
/* The whole exchange above in one collective call over a communicator (below: RCCL or a
 * transport; NULL = a single rank), every step's status agreed by all ranks: counts ->
 * set_layout -> queries/answer/apply -> claims/check_claims.  KETOGPU_ECOLLISION: every
 * rank reloads with another salt; KETOGPU_EINVAL: shared Subject.String() keys (R4). */
struct ketogpu_comm;
int ketogpu_shard_exchange(ketogpu_shard *s, struct ketogpu_comm *comm);
/* ketogpu_resolve_batch for a shard: ids of the requests' roots and targets this rank owns,
 * KETOGPU_NODE_NOT_OWNED for the others (the owner's answer is the one that counts);
 * status ENOTFOUND for wildcard roots (not evaluated partitioned), EINVAL nil subjects */
int ketogpu_shard_resolve_batch(const ketogpu_shard *s, const ketogpu_request_batch *reqs, uint32_t *roots,
                                uint32_t *targets, int32_t *status);
int ketogpu_shard_stats_get(const ketogpu_shard *s, ketogpu_shard_stats *out);
/* read-only view of the rank's device rows (tools, tests); global node ids */
typedef struct {
    uint32_t rank, world;
    uint32_t num_interior, num_expandable, num_nodes;       /* Ni, Nx, N (global)      */
    uint32_t owned_interior, owned_expandable, owned_nodes; /* local class bounds      */
    const uint64_t *lf_off; /* owned_expandable + 1: interior successors               */
    const uint32_t *lf_col;
    const uint64_t *lr_off; /* owned_nodes + 1: expandable predecessors, sorted          */
    const uint32_t *lr_col;
    const uint64_t *lb_off; /* owned_interior + 1: interior predecessors                */
    const uint32_t *lb_col;
} ketogpu_shard_graph;
int ketogpu_shard_view(const ketogpu_shard *s, ketogpu_shard_graph *out);

/* ------------------------------------------------------- partitioned mode */
/* Hash-partitioned traversal for graphs that do not fit one GPU (BASELINE config #5,
 * SURVEY.md 8(e)); replaces the same SubjectIsAllowed recursion as ketogpu_check_ids
 * (internal/check/engine.go:33-95), spread over ranks.  A rank's partition is its loaded
 * shard (ketogpu_shard_*): it holds the forward interior rows and traversal state of its
 * expandable nodes and the reverse rows of its nodes; ketogpu_part_owner(v) names the
 * rank that owns global node id v.  These
 * calls are one rank's device steps of a round; the caller moves the records between
 * ranks (keto_amd/partition.py: torch.distributed all_to_all over RCCL):
 *   begin -> { emit -> [all-to-all] -> apply -> [all-reduce frontier; stop at 0] -> expand }
 *         -> pull_emit -> [all-to-all] -> pull_answer -> end   (answer = OR of end() bits)
 * Buffers named *_dev are device memory on the rank's GPU.  A step that returns
 * KETOGPU_ENOMEM (buffers too small for this round) leaves the round to ketogpu_part_abort;
 * every rank must then abort and retry with fewer requests per round.  Snapshots with
 * ambiguous Subject.String() keys are refused (KETOGPU_EINVAL). */
typedef struct ketogpu_part ketogpu_part;
typedef struct {
    uint32_t a; /* BFS: 64-request word of the round; pull: request index of the round */
    uint32_t b; /* node id (global) — its owner receives the record                     */
    uint64_t m; /* BFS: request bits of word a; pull: 0                                  */
} ketogpu_record;
typedef struct {
    int32_t device;
    int32_t rank, world;          /* world <= 64                                       */
    uint64_t record_capacity;     /* outgoing records per step; 0 = auto               */
    uint32_t max_words_per_round; /* 0 = auto (state budget)                           */
    uint64_t state_budget_bytes;  /* 0 = auto                                          */
} ketogpu_part_opts;
/* kernel families of ketogpu_part_stats.ms / bytes / launches */
#define KETOGPU_PART_K_SEED 0
#define KETOGPU_PART_K_EXPAND 1
#define KETOGPU_PART_K_PACK 2        /* count + scatter by destination (world 1: a copy) */
#define KETOGPU_PART_K_APPLY 3
#define KETOGPU_PART_K_GATHER 4
#define KETOGPU_PART_K_PULL_EMIT 5
#define KETOGPU_PART_K_PULL_ANSWER 6
#define KETOGPU_PART_K_RESET 7
typedef struct {
    uint64_t owned_interior, owned_expandable, owned_forward_edges, owned_reverse_edges;
    uint64_t rounds, levels, frontier_entries, forward_edges;
    uint64_t records_sent, records_received, queries_answered;
    /* per kernel family: algorithmic HBM bytes (always counted) and, while timing is on
     * (ketogpu_part_set_timing), summed hipEvent device time and timed launches */
    uint64_t bytes[8];
    double ms[8];
    uint64_t launches[8];
} ketogpu_part_stats;
/* opts->rank / world must match the shard's */
int ketogpu_part_new(const ketogpu_shard *s, const ketogpu_part_opts *opts, ketogpu_part **out);
uint32_t ketogpu_part_owner(const ketogpu_part *p, uint32_t node);
void ketogpu_part_free(ketogpu_part *p);
/* 64-request words one round holds */
uint64_t ketogpu_part_round_words(const ketogpu_part *p);
/* same (roots, targets) host arrays on every rank, n <= 64 * round_words */
int ketogpu_part_begin(ketogpu_part *p, const uint32_t *roots, const uint32_t *targets, size_t n);
/* Same round, in a chosen direction (partition.hip header): KETOGPU_PART_FORWARD grows the
 * roots' closures X(r) (what ketogpu_part_begin does), KETOGPU_PART_BACKWARD grows the
 * targets' ancestor sets B(t) along interior-predecessor rows and pulls from the roots'
 * rows.  Same answers; every rank must use the same direction in a round. */
#define KETOGPU_PART_FORWARD 0
#define KETOGPU_PART_BACKWARD 1
int ketogpu_part_begin_dir(ketogpu_part *p, const uint32_t *roots, const uint32_t *targets, size_t n,
                           int32_t direction);
/* this step's outgoing records grouped by destination rank into send_dev; counts[world].
   world > 1: send_dev is complete on return (any stream may read it).  world == 1: the copy
   is ordered on the partition's stream only; pass send_dev straight to ketogpu_part_apply /
   _pull_answer (which run on that stream) or call ketogpu_part_sync first. */
int ketogpu_part_emit(ketogpu_part *p, ketogpu_record *send_dev, uint64_t capacity, uint64_t *counts);
/* OR received records into the owned state; *frontier = owned entries of the next level */
int ketogpu_part_apply(ketogpu_part *p, const ketogpu_record *recv_dev, uint64_t n, uint64_t *frontier);
/* the owned frontier's rows -> the next emit's records */
int ketogpu_part_expand(ketogpu_part *p);
/* after the last level: direct hits of owned targets + queries (request, interior node) */
int ketogpu_part_pull_emit(ketogpu_part *p, ketogpu_record *send_dev, uint64_t capacity, uint64_t *counts);
int ketogpu_part_pull_answer(ketogpu_part *p, const ketogpu_record *recv_dev, uint64_t n);
/* this rank's hit bits of the round (ceil(n/64) host words) and state reset */
int ketogpu_part_end(ketogpu_part *p, uint64_t *allowed_bits);
int ketogpu_part_abort(ketogpu_part *p);
/* wait for the partition's stream (world 1: makes the last emit's send_dev readable elsewhere) */
int ketogpu_part_sync(ketogpu_part *p);
int ketogpu_part_stats_get(const ketogpu_part *p, ketogpu_part_stats *out);
/* on: every kernel launch of the partition is bracketed by hipEvents on its stream (a
 * measurement pass; each event costs a few microseconds of GPU idle) */
int ketogpu_part_set_timing(ketogpu_part *p, int32_t on);

/* --------------------------------------------- partitioned mode: whole rounds */
/* The same rounds as above with the exchange inside the library, so a Go host drives a
 * hash-partitioned PermissionEngine through ONE call per batch, like ketogpu_check_ids
 * (the engine is built once per process, internal/driver/registry_default.go:158-163;
 * SubjectIsAllowed's recursion, internal/check/engine.go:33-95, spread over ranks).
 *
 * A communicator joins the ranks of one partitioned network (one process per GPU):
 *   RCCL over xGMI  rank 0: ketogpu_comm_unique_id(id); broadcast id to every rank out of
 *                   band (a Go host: its own channel; tests: torch.distributed); then every
 *                   rank ketogpu_comm_new(id, rank, world, device) (ncclCommInitRank,
 *                   /opt/rocm/include/rccl/rccl.h:220).  Records are exchanged from device
 *                   memory on the partition's stream: grouped ncclSend/ncclRecv per peer
 *                   (rccl.h:700-725), counts and statuses by ncclAllGather.
 *   a transport     ketogpu_comm_from_transport(vtable): the caller moves host bytes (a Go
 *                   transport; the CPU tests use torch.distributed gloo).
 * Per BFS level every rank makes one small all-gather (each rank's per-destination record
 * counts plus its step status — a step that failed anywhere fails the round everywhere,
 * and a level where no rank sends anything ends the closure: no depth cutoff, R2) and one
 * all-to-all of the records; a round ends with one all-gather of the ranks' hit bits (the
 * answer is their OR).  Every rank calls ketogpu_part_check_ids with the same requests and
 * gets the full answer.  Rounds whose buffers overflow are retried with half the requests
 * on every rank; KETOGPU_PART_AUTO times one round in each direction (max over ranks, so
 * every rank decides alike) and keeps the faster. */
typedef struct ketogpu_comm ketogpu_comm;
#define KETOGPU_COMM_ID_BYTES 128
int ketogpu_comm_unique_id(uint8_t id[KETOGPU_COMM_ID_BYTES]);
int ketogpu_comm_new(const uint8_t id[KETOGPU_COMM_ID_BYTES], int32_t rank, int32_t world, int32_t device,
                     ketogpu_comm **out);
#define KETOGPU_REDUCE_MIN 0
#define KETOGPU_REDUCE_MAX 1
/* host-memory transport; every callback returns 0 on success.  Collective: every rank
 * calls the same callbacks in the same order. */
typedef struct {
    void *ctx;
    int32_t rank, world;
    /* every rank's `bytes` -> recv (world * bytes, rank order) */
    int (*allgather)(void *ctx, const void *send, void *recv, uint64_t bytes);
    /* send grouped by destination (send_bytes[world]) -> recv grouped by source
       (recv_bytes[world], known to the caller) */
    int (*alltoallv)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv,
                     const uint64_t *recv_bytes);
    /* n u32 values reduced elementwise in place (KETOGPU_REDUCE_MIN / _MAX) */
    int (*allreduce_u32)(void *ctx, uint32_t *buf, uint64_t n, int32_t op);
} ketogpu_transport;
int ketogpu_comm_from_transport(const ketogpu_transport *t, ketogpu_comm **out);
void ketogpu_comm_free(ketogpu_comm *c);
/* RCCL calls a communicator made (counts since creation; a host transport's are 0).
 * KETOGPU_TEST_RCCL_SELF=1 when an RCCL communicator is made (tests): at world 1 too, the
 * all-to-alls move the rank's own segment with a grouped ncclSend/ncclRecv to itself and
 * the two-tier count gathers run as ncclAllGather, so one GPU executes the multi-GPU
 * data path (default: the own segment is a copy-engine DMA and world-1 gathers are skipped) */
typedef struct {
    int32_t rccl, loop_self;
    uint64_t sends, recvs, allgathers, allreduces, bytes_sent;
} ketogpu_comm_stats;
int ketogpu_comm_stats_get(const ketogpu_comm *c, ketogpu_comm_stats *out);
int ketogpu_comm_rank(const ketogpu_comm *c);
int ketogpu_comm_world(const ketogpu_comm *c);

/* ketogpu_shard_resolve_batch combined over the ranks (the owners' answers win):
 * status ENOTFOUND = a wildcard root (R5), which the partitioned engine does not evaluate;
 * EINVAL = nil subject.  comm NULL: a single rank. */
int ketogpu_part_resolve_batch(const ketogpu_shard *s, ketogpu_comm *c, const ketogpu_request_batch *reqs,
                               uint32_t *roots, uint32_t *targets, int32_t *status);

typedef struct ketogpu_part_engine ketogpu_part_engine;
#define KETOGPU_PART_AUTO (-1)
typedef struct {
    int32_t direction;        /* KETOGPU_PART_FORWARD, _BACKWARD or _AUTO                  */
    uint64_t record_capacity; /* records per exchange buffer; 0 = the partition's own      */
} ketogpu_part_engine_opts;
/* comm NULL: world 1 without any exchange (records stay where the kernels wrote them).
 * The engine borrows p and c (free it first). */
int ketogpu_part_engine_new(ketogpu_part *p, ketogpu_comm *c, const ketogpu_part_engine_opts *opts,
                            ketogpu_part_engine **out);
/* one batch: every rank passes the same requests (host memory), n any size; allowed_bits
 * ceil(n/64) words */
int ketogpu_part_check_ids(ketogpu_part_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                           uint64_t *allowed_bits);
typedef struct {
    int32_t direction;          /* the kept direction (KETOGPU_PART_AUTO before any round) */
    uint64_t trial_ns[2];       /* auto: ns per request of each direction's trial round     */
    uint64_t rounds, levels;    /* rounds run (trials and retries included), BFS levels     */
    uint64_t records_sent, records_received, retries, collectives;
    double exchange_ms;         /* host wall time inside collectives                        */
} ketogpu_part_engine_stats;
int ketogpu_part_engine_stats_get(const ketogpu_part_engine *e, ketogpu_part_engine_stats *out);
void ketogpu_part_engine_free(ketogpu_part_engine *e);

/* Test hook: the same driver over caller-provided steps in host memory (the CPU tests
 * play a rank's device steps with them, tests/part_cpu.py; the product passes a
 * ketogpu_part).  Callbacks mirror ketogpu_part_begin_dir / _emit (pull = 0) /
 * _pull_emit (pull = 1) / _apply / _expand / _pull_answer / _end / _abort. */
typedef struct {
    void *ctx;
    uint64_t round_words;
    int (*begin)(void *ctx, const uint32_t *roots, const uint32_t *targets, uint64_t n, int32_t direction);
    int (*emit)(void *ctx, int32_t pull, ketogpu_record *send, uint64_t capacity, uint64_t *counts);
    int (*apply)(void *ctx, const ketogpu_record *recv, uint64_t n, uint64_t *frontier);
    int (*expand)(void *ctx);
    int (*pull_answer)(void *ctx, const ketogpu_record *recv, uint64_t n);
    int (*end)(void *ctx, uint64_t *allowed_bits);
    int (*abort)(void *ctx);
} ketogpu_part_steps;
int ketogpu_part_engine_new_steps(const ketogpu_part_steps *steps, ketogpu_comm *c,
                                  const ketogpu_part_engine_opts *opts, ketogpu_part_engine **out);

/* ------------------------------------------- partitioned mode: two-tier */
/* The same hash-partitioned network (ketogpu_shard_*) checked with TWO exchanges per batch
 * instead of two per BFS level, when its CORE fits every GPU.  The core is the rows among
 * interior nodes: fint(v) and the interior predecessors of every interior node v (group
 * nesting: ~0.3% of config #5's tuples).  Every path r -> v1 -> ... -> t of the reference's
 * recursion (internal/check/engine.go:33-91) has v1 in fint(r), its last interior node in
 * rev(t) and everything between inside the core, so each rank keeps a copy of the core and
 * only the two seed rows of a request live elsewhere:
 *   queries  request i asks owner(r) for fint(r) and owner(t) for rev(t)  [all-to-all]
 *   replies  the owners send those rows                                     [all-to-all]
 *   evaluate the bidirectional LDS unit of the single-GPU engine over the local core
 * (plan label, the default: the owners reply with their nodes' 2-hop label lists instead
 * and the evaluation is one list intersection per request)
 * A world of one rank reads its own rows in place (no exchange at all).  Unlike
 * ketogpu_part_check_ids, every rank passes ITS OWN requests (any number, 0 included)
 * and gets the answers to them; the call is collective (every rank calls it for each of
 * its batches, as with the per-level engine).  Requests whose search outgrows the LDS
 * tables (none on the benchmark graphs) are answered by the per-level engine, built on
 * first need from the same shard and communicator.  Same answers as ketogpu_check_ids on
 * the whole graph (the R2 formula, no depth cutoff).
 *
 *   ketogpu_core_gather (collective, once per load) -> ketogpu_tier_new -> check_ids ...
 *
 * ketogpu_core_gather fails with KETOGPU_ENOMEM on every rank alike when the core passes
 * core_budget_bytes (the per-level engine is then the partitioned mode to use). */
typedef struct ketogpu_core ketogpu_core;
typedef struct {
    uint32_t num_interior;     /* Ni: core rows                                          */
    const uint64_t *f_off;     /* Ni + 1: interior successors of each interior node      */
    const uint32_t *f_col;
    const uint64_t *b_off;     /* Ni + 1: interior predecessors of each interior node    */
    const uint32_t *b_col;
    uint64_t bytes;            /* device bytes of the core's records                     */
} ketogpu_core_view;
/* opts: the shard's; comm NULL for a single rank.  core_budget_bytes 0: no limit here */
int ketogpu_core_gather(const ketogpu_shard *s, ketogpu_comm *comm, uint64_t core_budget_bytes, ketogpu_core **out);
int ketogpu_core_get_view(const ketogpu_core *c, ketogpu_core_view *out);
void ketogpu_core_free(ketogpu_core *c);

typedef struct ketogpu_tier ketogpu_tier;
typedef struct {
    int32_t device;
    uint64_t max_batch;            /* requests evaluated per step; 0 = 4M                */
    uint64_t fallback_state_bytes; /* the per-level engine's state budget; 0 = 2 GB      */
} ketogpu_tier_opts;
/* a request's query in transit: tag = request index << 1 | 0 (fint(r)) / 1 (rev(t)) */
typedef struct {
    uint32_t tag, node;
} ketogpu_tier_query;
/* a row entry in transit: the entry's node and its request's tag (the receiver looks the
 * entry's core row up in its own copy of the core) */
typedef struct {
    uint32_t node, tag;
} ketogpu_tier_rec;
typedef struct {
    uint64_t calls, batches, requests, overflow_requests, fallback_calls;
    uint64_t queries_sent, records_sent, records_received, collectives;
    uint64_t rows_opened, records_read; /* device statistics of the evaluation      */
    double exchange_ms, evaluate_ms;    /* host wall time inside collectives / evaluation */
    uint64_t core_records, seed_records; /* device records: core (both directions), own rows */
    double eval_kernel_ms;               /* hipEvent time of the first evaluation stage      */
    uint64_t eval_kernel_launches;
    /* plan label (KETOGPU_TIER_LABEL=0 at ketogpu_tier_new: off): owners answer a query with
     * the node's label list (masks + entries) instead of its row, and the evaluation is one
     * intersection per request (no later stage, no per-level fallback).  rows_opened: 2 per
     * request, records_read: list words read */
    uint64_t label;                      /* 1: plan label                                    */
    uint64_t label_words;                /* this rank's S and P list words (masks included)  */
    double label_build_ms;               /* labels of the core + the owned lists             */
} ketogpu_tier_stats;
/* the shard and core stay owned by the caller; the tier borrows s, core and comm */
int ketogpu_tier_new(const ketogpu_shard *s, const ketogpu_core *core, ketogpu_comm *comm,
                     const ketogpu_tier_opts *opts, ketogpu_tier **out);
/* this rank's n requests (host memory — pinned buffers are read in place — or the tier
 * device's memory, read in place by every pass) -> ceil(n/64) words of answer bits (host
 * memory).  An id outside the layout fails the call with
 * KETOGPU_EINVAL on that rank (its peers fail with the same code). */
int ketogpu_tier_check_ids(ketogpu_tier *t, const uint32_t *roots, const uint32_t *targets, size_t n,
                           uint64_t *allowed_bits);
int ketogpu_tier_stats_get(ketogpu_tier *t, ketogpu_tier_stats *out);
void ketogpu_tier_free(ketogpu_tier *t);
/* Test hook: the same protocol over caller steps in host memory (tests/tier_cpu.py).
 * queries: this rank's requests -> queries grouped by owner (counts[world]);
 * reply_sizes: received queries (grouped by source, from[world] each) -> records per
 * destination (counts[world]); reply_emit: those records, in query order;
 * evaluate: the answers (recv NULL: the rank owns every row, world 1) and the indices of
 * requests it could not finish (overflow; none for host steps). */
typedef struct {
    void *ctx;
    int (*queries)(void *ctx, const uint32_t *roots, const uint32_t *targets, uint64_t n, ketogpu_tier_query *send,
                   uint64_t *counts);
    int (*reply_sizes)(void *ctx, const ketogpu_tier_query *recv, uint64_t n, const uint64_t *from,
                       uint64_t *counts);
    int (*reply_emit)(void *ctx, ketogpu_tier_rec *send);
    int (*evaluate)(void *ctx, const uint32_t *roots, const uint32_t *targets, uint64_t n,
                    const ketogpu_tier_rec *recv, uint64_t nrecv, uint64_t *allowed_bits, uint32_t *overflow,
                    uint64_t *n_overflow);
} ketogpu_tier_steps;
int ketogpu_tier_new_steps(const ketogpu_tier_steps *steps, ketogpu_comm *comm, const ketogpu_tier_opts *opts,
                           ketogpu_tier **out);

/* ------------------------------------------------------------------ expand */
/* BuildTree(subject, rest_depth).  *out = NULL is the nil tree (JSON null).
 * KETOGPU_ENOTFOUND when a fetched page references an unknown namespace. */
int ketogpu_expand(const ketogpu_snapshot *s, const ketogpu_subject *subject, int32_t rest_depth,
                   ketogpu_tree **out);

#define KETOGPU_NODE_UNION 0
#define KETOGPU_NODE_LEAF 1
/* flattened tree in preorder; strings are owned by the tree */
typedef struct {
    int32_t type;         /* KETOGPU_NODE_UNION / KETOGPU_NODE_LEAF                */
    uint32_t num_children;/* the children follow in preorder                      */
    ketogpu_subject subject;
} ketogpu_tree_node;
int ketogpu_tree_nodes(const ketogpu_tree *t, const ketogpu_tree_node **nodes, size_t *n);
/* MarshalJSON of the tree (tree.go:156-162); free with ketogpu_free */
int ketogpu_tree_json(const ketogpu_tree *t, char **json);
void ketogpu_tree_free(ketogpu_tree *t);

/* ------------------------------------------------------------------- misc */
const char *ketogpu_last_error(void);
int ketogpu_abi_version(void);
void ketogpu_free(void *p);
/* number of visible HIP devices (0 without a GPU) */
int ketogpu_device_count(void);
/* diagnostics (no Keto counterpart): the random-line ceiling of plan label's first stage —
 * `requests` requests of 16 per wave each reading two random 128-byte lines of a
 * `table_bytes` table plus 8 bytes of request, the reads a check of plan label makes and
 * nothing else; *ms_per_launch averaged over `reps` launches on `device` (keto_amd/csrc/
 * probe.hip; bench.py's roofline.line_ceiling) */
int ketogpu_probe_random_lines(int device, uint64_t table_bytes, uint64_t requests, int reps, double *ms_per_launch);

#ifdef __cplusplus
}
#endif
#endif
