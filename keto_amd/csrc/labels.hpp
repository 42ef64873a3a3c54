// labels.hpp — the reachability labels of plan "label" (device_engine.hip label_unit).
//
// The reference answers a check by the recursion of internal/check/engine.go:33-91; for a
// request (r, t) that is R2 reachability (semantic contract): some row path
// r -> x1 -> ... -> t whose inner nodes are INTERIOR.  Plan label answers it with ONE
// intersection of two short sorted lists per request, whatever the graph's shape.
//
// 2-hop labels of the interior graph (pruned landmark labeling): interior nodes are ranked
// (most central first) and every node v gets Lin(v) = landmarks w with w ->* v and
// Lout(v) = landmarks w with v ->* w, such that for interior a, b
//     a ->* b (reflexive)  <=>  Lout(a) and Lin(b) share a landmark.
// The first kMaskBits landmarks are kept as a bit mask per node instead of list entries
// (min / mout: bit i = landmark i reaches the node / the node reaches landmark i); the
// others are processed in rank order, each a forward and a backward search that stops at
// nodes the labels built so far already answer (landmarks of one parallel batch do not
// prune each other: more entries, never a wrong answer).
//
// Per request, with rev(t) the expandable nodes whose rows hold t and fint(r) r's interior
// successors:
//   S(t) = Lin(v) for every interior v in rev(t)  +  raw(t), the non-interior entries of rev(t)
//   P(r) = Lout(r)                                  (r interior)
//        = Lout(c) for every c in fint(r)           (r expandable, not interior)
//   allowed(r, t)  <=>  P(r) and S(t) share a landmark (or their masks share a bit)
//                       or  r is not interior and r in raw(t)          (the one-edge test)
// Proof: a path's last inner node v is in rev(t) and its first one c in fint(r) (c = v
// possible), so c ->* v; r interior: r ->* v; a one-edge path has r in rev(t) (r interior:
// r ->* r, so Lin(r) in S(t) meets Lout(r); r not interior: r in raw(t)).  Conversely a shared
// landmark w gives r (->c) ->* w ->* v -> t, and r in raw(t) is the edge r -> t.  Landmark
// entries are RANKS (< Ni) and raw entries node ids (>= Ni): a sorted S list is its landmarks
// then its raw entries, and a landmark never equals a raw entry or a non-interior root.
//
// Storage (u32 words), one fixed-size HEAD per node (S: every node, P: every expandable
// node), hs / hp words each (8, 16, 32 or 64, labels.cpp pick_head):
//   [count | overflow start / 16 | mask lo | mask hi | entries ascending ... | 0xFFFFFFFF pad]
// a list of more than head - 4 entries is kept whole at words 16 x (overflow start) (after
// the heads, in the same array), its first head - 4 entries also in the head; count =
// kNoLabel: the request goes to the second stage.  An S head's count is its whole list
// (landmarks and raw entries); where its landmarks end is found among the entries (the
// first entry >= Ni).
//
// The first stage (device_engine.hip label_unit) decides a request from the two heads alone
// when it can: a hit among the masks, the inline landmark prefixes or (r not interior) the
// inline raw entries; else "denied" when no landmark can be missing from the prefixes — both
// landmark lists whole in their heads, or one whole with its largest entry <= the other's
// last inline entry (a common landmark would then lie in both prefixes) — and the raw test
// is settled (r interior, S whole in its head, or r <= its last inline entry).  Otherwise
// the dense pass reads the overflow lists.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "ketogpu_internal.hpp"

namespace ketogpu {

constexpr uint32_t kNoLabel = 0xFFFFFFFFu;
constexpr uint32_t kMaskBits = 64;   // landmarks kept as a bit mask
constexpr uint32_t kHeadFixed = 4;   // count, overflow start, mask (2 words)

// the 2-hop labels of the interior graph
struct ReachLabels {
    uint32_t n = 0;                      // interior nodes
    uint32_t bits = 0;                   // landmarks in the masks (min(n, kMaskBits))
    std::vector<uint32_t> order;         // rank -> interior node
    std::vector<uint64_t> min, mout;     // per node
    std::vector<uint64_t> in_off, out_off;
    std::vector<uint32_t> in, out;       // ranks >= bits, ascending per node
    uint64_t batches = 0;                // parallel batches of the pruned searches
    uint64_t version = 0;                // the snapshot version they were built at
    double ms = 0;
};

// KETOGPU_LABEL_SEQ: landmarks searched one at a time after the masked ones (default 0);
// the others run in parallel batches of max(4 x threads, rank / KETOGPU_LABEL_BATCH_DIV)
// (default 8)
void build_reach_labels(const Snapshot &s, ReachLabels &out);
// the same over a graph given as CSR rows (n nodes; forward and backward rows, every entry
// below n): the two-tier partitioned mode's replicated core (tier.cpp)
void build_reach_labels_csr(uint32_t n, const uint64_t *f_off, const uint32_t *f_col, const uint64_t *b_off,
                            const uint32_t *b_col, ReachLabels &out);
// the interior graph as CSR copies (a writable snapshot: its real entries only, as
// build_reach_labels sees them): what a background relabel builds from while the snapshot
// keeps taking writes (device_engine.hip start_relabel)
struct InteriorCsr {
    uint32_t n = 0;
    std::vector<uint64_t> f_off, b_off;
    std::vector<uint32_t> f_col, b_col;
};
void copy_interior(const Snapshot &s, InteriorCsr &out);
// the snapshot's labels, built once per snapshot version and shared by every engine over
// it (ketogpu_multi_new builds one set for all devices)
std::shared_ptr<const ReachLabels> reach_labels_of(const Snapshot &s);

// one node's list and mask as its head holds them (p_side: P(x), else S(x))
void label_list(const Snapshot &s, const ReachLabels &R, bool p_side, uint64_t x, std::vector<uint32_t> &out,
                uint64_t &mask);
// the head size from the list lengths; fit[k]: non-empty lists of at most (8 << k) - 4
// entries (k = 0..3: heads of 8, 16, 32, 64 words).  A random head read costs one 128-byte
// line whether the head has 8, 16 or 32 words (profiles/r06/probe), a 64-word head two, about
// what the dense pass spends on 8-10% of the requests (config #2, round 5): 64 words when
// they hold >= 10% more of the non-empty lists inline than 32 words, else the smallest of 8,
// 16, 32 words that holds (within 0.1%) as many lists inline as 32 words
uint32_t pick_head(uint64_t nonempty, const uint64_t fit[4]);
// S heads: every node, and on a writable snapshot every reserved id too (n_cap)
uint64_t label_s_nodes(const Snapshot &s);
// the KETOGPU_LABEL_REST_PERMILLE test knob: S head of x marked kNoLabel
bool label_nolabel(uint64_t x, uint32_t permille);

struct LabelIndex {
    uint32_t hs = 16, hp = 8;            // head words of S and P (8, 16, 32 or 64)
    std::vector<uint32_t> S, P;          // heads then overflow lists
    uint64_t s_nodes = 0, p_nodes = 0;
    uint64_t s_entries = 0, p_entries = 0;    // list entries (masks not counted)
    uint64_t s_overflow = 0, p_overflow = 0;  // lists kept outside their head
    uint64_t s_nolabel = 0;                   // heads marked kNoLabel (test knob)
    uint64_t label_entries = 0;               // Lin + Lout entries
    double pll_ms = 0, build_ms = 0;
};

// Builds the labels and both head arrays.  hs / hp = 0: chosen from the list lengths.
// rest_permille > 0 (test knob): that share of the S heads (by node hash) is marked
// kNoLabel.  max_bytes: the arrays must fit (KETOGPU_ENOMEM before anything is allocated
// otherwise).
void build_labels(const Snapshot &s, uint32_t hs, uint32_t hp, uint32_t rest_permille, uint64_t max_bytes,
                  LabelIndex &out);

}  // namespace ketogpu
