// labels.hpp — closure labels of plan "label" (device_engine.hip label_unit).
//
// The reference answers a check by the recursion of internal/check/engine.go:33-91; for a
// request (r, t) that is R2 reachability: some row path r -> x1 -> ... -> t whose inner
// nodes are interior (semantic contract).  With the closure rows of plan core
// (core_index.hpp) that reachability becomes ONE intersection of two short lists per
// request, in either of two modes:
//   mode B (backward label):  P(r) = {r} + fint(r),  S(t) = rev(t) + Anc+(g) for every
//                             interior g in rev(t)       allowed <=> P(r) meets S(t)
//   mode F (forward label):   P(t) = rev(t),          S(r) = {r} + fint(r) + Desc+(h) for
//                             every h in fint(r)         allowed <=> P(t) meets S(r)
// (a path's first interior node x1 is in fint(r) and its last one in rev(t); x1 reaches
// x(k-1) through interior nodes, so x1 is in Anc+(x(k-1)) and x(k-1) in Desc+(x1); a path
// of one edge has r in rev(t)).  S is a LABEL: stored sorted per node when every closure it
// needs exists and it has at most s_words - 1 nodes; a request whose S is missing is
// answered by plan core's traversal instead (a second stage over those requests).
//
// Storage, per mode, all u32 words:
//   S blocks, one per S node (s_words = 64 or 128 words, 256 / 512 bytes, aligned): [count,
//     entries sorted ascending, 0xFFFFFFFF padding]; count = 0xFFFFFFFF: no label
//   P blocks, one per P node (pb words): [count, overflow start, entries...]; a row of more
//     than pb - 2 entries keeps the rest at p[overflow start ...] (an overflow region after
//     the blocks, in the same array)
#pragma once

#include <cstdint>
#include <vector>

#include "core_index.hpp"

namespace ketogpu {

constexpr uint32_t kNoLabel = 0xFFFFFFFFu;

struct LabelIndex {
    int mode = -1;                 // 0 = B, 1 = F; -1: not built
    uint32_t s_words = 64;         // S block words (64 or 128: labels of up to 63 or 127 nodes)
    uint32_t pb = 0;               // P block words
    std::vector<uint32_t> P, S;
    uint64_t p_nodes = 0, s_nodes = 0;
    uint64_t covered = 0;          // S nodes with a label (of those with a non-empty row)
    uint64_t nonempty = 0;
    double coverage[2] = {0, 0};   // per mode: labelled share of the S nodes with a non-empty row
    double build_ms = 0;
};

// mode: 0 / 1 forces B / F, -1 builds the mode whose labels cover more S nodes (none when
// both cover less than min_coverage).  Needs the closure rows of ci (build_core_index).
void build_labels(const Snapshot &s, const CoreIndex &ci, int mode, double min_coverage, LabelIndex &out,
                  uint32_t s_words = 64);

}  // namespace ketogpu
