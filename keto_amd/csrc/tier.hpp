// tier.hpp — the two-tier partitioned mode (internal; include/ketogpu.h "two-tier").
//
// A hash-partitioned network (shard.cpp) whose CORE — the rows among interior nodes:
// fint(v) and the interior predecessors of every interior node v — is small enough to be
// copied to every rank, while the bulk of the rows (a document's grants, a user's
// memberships: every row that starts or ends outside the interior) stays with its owner.
// Every path r -> v1 -> ... -> v(k-1) -> t has v1 in fint(r), v(k-1) in rev(t) and
// everything between in the core, so a check needs exactly two rows from the owners —
// fint(r) from owner(r), rev(t) from owner(t) — and then runs the bidirectional LDS unit
// (device_engine.hip lite_unit) on the local copy of the core, with no exchange per level.
// The kernels live in device_engine.hip (they share lite_unit); the host state and the
// exchange protocol in tier.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ketogpu_internal.hpp"

namespace ketogpu {

// device_engine.hip: `device`'s view of host memory it can read in place (pinned), else
// nullptr
// is_device (may be null): set when p is memory of `device` itself (HBM)
const void *host_view(const void *p, int device, bool query, bool *is_device = nullptr);

namespace tier {

// a 16-byte edge record (device_engine.hip FRec): the entry's node, the entry's own core
// row (forward: |fint(node)| and its first record; backward: |interior predecessors of
// node| and its first record; 0/0 for a backward entry outside the interior), pad (in
// transit: the request tag)
struct Rec {
    uint32_t node, deg, begin, pad;
};
// a query in transit: tag = request index << 1 | direction (0: fint(r), 1: rev(t))
struct Query {
    uint32_t tag, node;
};
// a reply entry in transit (include/ketogpu.h ketogpu_tier_rec): 8 bytes; the receiver
// turns it into a Rec with its own copy of the core
struct Reply {
    uint32_t node, tag;
};

// device view of one rank's graph
struct Graph {
    uint32_t world, rank, Ni, Nx, N;  // global layout (shard.cpp)
    uint32_t Nil, Nxl, Nl;            // owned class bounds
    const Rec *core_f, *core_b;       // core rows of every interior node (replicated)
    const uint2 *core_f_row, *core_b_row;  // [Ni] {first record, count}: a received entry's core row
    const uint64_t *lf_off, *lr_off;  // owned seed rows: fint of owned expandable, rev of owned nodes
    const Rec *lf_rec, *lr_rec;
    const uint32_t *lf_node, *lr_node;  // the same rows' entries as plain node ids (the replies)
    int64_t lf_base, lr_base;         // lf_rec - core_f and lr_rec - core_b in records
    uint32_t both_max, seed_max;
    // label mode (plan label, labels.hpp): every rank builds the same 2-hop labels of the
    // replicated core; an owner's S list of every owned node and P list of every owned
    // expandable node, each [mask lo, mask hi, entries ascending]: a query is answered with
    // the list instead of the row, and the evaluation is one intersection per request
    uint32_t label;
    const uint64_t *ls_off, *lp_off;
    const uint32_t *ls_col, *lp_col;
};

// evaluation stages: 0 = one 16-request unit per workgroup over every unit of the batch,
// 1 / 2 = persistent cascades over the previous stage's spilled units (larger tables)
constexpr int kStages = 3;
// bnd: per request {fb, fe, rb, re} into recv (exchange mode), or nullptr: the rank owns
// every root and target and reads the seed rows in place (world 1)
struct Eval {
    const uint32_t *roots, *targets;  // device-readable (HBM or a pinned host view)
    uint64_t n;
    const uint4 *bnd;
    const Rec *recv;
    int64_t recv_base_f, recv_base_b;  // recv - core_f, recv - core_b in records
    uint64_t *allowed;                 // ceil(n/64) words, cleared by the caller
    unsigned long long *stats;         // [0] rows opened, [1] records read
    unsigned long long *first_bad;     // lowest invalid request index (~0: none)
};
void launch_eval(int stage, const Graph &g, const Eval &e, const uint32_t *in_list, const unsigned *in_count,
                 uint32_t *out_list, unsigned *out_count, unsigned grid, hipStream_t s);
// Label replies (plan label): 4-byte words; the segment for one destination is the lengths
// of the lists it asked for (its query order), then the lists.  With qs[p] the first query
// of segment p (p = 0..world, qs[world] = total) and off the lengths' exclusive scan over
// all queries, query j of segment p has its length at j + off[qs[p]] and its list at
// qs[p + 1] + off[j] — the same formula on the asking side over ITS sent queries.
//   owner:  reply_lengths -> scan -> launch_label_reply (lengths and lists in one pass)
//   asker:  launch_label_lens (the lengths out of the received segments, rp[p] = segment
//           p's first word) -> scan -> launch_label_bounds (per request the bounds of its P
//           list (x, y) and S list (z, w); bnd cleared by the caller; a list ending past
//           cap received words: left empty) -> launch_label_eval
// launch_label_eval: recv_label null: the rank owns every node and reads its own lists; the
// answer array needs no clearing (each unit stores its 16-bit word); world 1: qs not read
// bnd (world 1, else null): the replies' own bounds per request, written by the same pass
// srcb: each list's first word in lp_col / ls_col (launch_reply_lengths)
void launch_label_reply(const Graph &g, const Query *q, uint64_t n, const uint64_t *off, const uint64_t *srcb,
                        const uint64_t *qs, uint32_t world, uint32_t *out, uint64_t cap, uint4 *bnd, uint64_t nreq,
                        hipStream_t s);
void launch_label_lens(const uint32_t *recv, uint64_t nsent, const uint64_t *sq, const uint64_t *rp, uint32_t world,
                       uint64_t *lens, hipStream_t s);
void launch_label_bounds(const Query *sent, uint64_t nsent, const uint64_t *sq, const uint64_t *g, uint32_t world,
                         uint4 *bnd, uint64_t nreq, uint64_t cap, hipStream_t s);
void launch_label_eval(const Graph &g, const Eval &e, const uint32_t *recv_label, hipStream_t s);
int stage_units_per_cu(int stage);

// queries of the batch grouped by owner: count (per destination) then scatter at cursors
// stage (may be null): the requests are also copied there (2n words: roots, then targets),
// so later passes read them from HBM instead of host memory again
void launch_query_count(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n,
                        unsigned long long *counts, unsigned long long *first_bad, uint32_t *stage, hipStream_t s);
// world 1: request i's queries at slots 2i, 2i + 1 (NONE nodes: no answer); no counting
void launch_query_pairs(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n, Query *out,
                        unsigned long long *first_bad, uint32_t *stage, hipStream_t s);
void launch_query_scatter(const Graph &g, const uint32_t *roots, const uint32_t *targets, uint64_t n,
                          unsigned long long *cursor, Query *out, hipStream_t s);
// replies: the rows the received queries ask for, in query order (so grouped like the
// queries' sources); `lens` scratch of n + 1 entries, *total the number of records
// (device word), written with pad = the query's tag
// srcb (may be null): each row's / list's first entry (label replies read it back)
void launch_reply_lengths(const Graph &g, const Query *q, uint64_t n, uint64_t *lens, unsigned long long *bad,
                          hipStream_t s, uint64_t *srcb = nullptr);
// answers into the caller's pinned words (bits may be null) and the status words into the
// steps' pinned ones, one launch (tier_emit_kernel)
// (status reset to ~0 once copied)
void launch_emit(const uint64_t *allowed, uint64_t words, uint64_t *bits, unsigned long long *status,
                 const uint64_t *total, unsigned long long *h_status, uint64_t *h_total, hipStream_t s);
void launch_scan(uint64_t *v, uint64_t n, uint64_t *scratch, hipStream_t s);  // exclusive, in place, v[n] = total
void launch_reply_copy(const Graph &g, const Query *q, uint64_t n, const uint64_t *off, Reply *out, uint64_t cap,
                       hipStream_t s);
// received replies -> seed records (the entries' core rows looked up) and per request seed
// bounds (bnd cleared by the caller), one pass
void launch_seed_records(const Graph &g, const Reply *recv, uint64_t n, Rec *seed, uint4 *bnd, uint64_t nreq,
                         hipStream_t s);

}  // namespace tier
}  // namespace ketogpu
