// core_index.hpp — the record arrays of plan "core" (device_engine.hip, lite_unit<CL>).
//
// Every check path r -> v1 -> ... -> v(k-1) -> t of the reference's recursion
// (internal/check/engine.go:33-91) starts with a row of r's (fint(r)), ends with a row
// containing t (rev(t)) and runs among INTERIOR nodes in between.  Plan "core" keeps the
// rows among interior nodes (the core) in two small record arrays of their own, and adds
// CLOSURE ROWS: for an interior node v whose forward closure Desc+(v) (interior nodes v
// reaches through >= 1 edge) or backward closure Anc+(v) (interior nodes that reach v) has
// at most `cap` nodes, the record that expands v in that direction points at the closure
// instead of v's one-hop row.  Pushing the closure marks every node of it visited at once
// (TERMINAL entries: visited, never pending), so a search side made of closure rows is
// complete after ONE level instead of one level per hop.  Exact for R2 reachability:
// every node of a closure is reachable from (reaches) v, and every node reachable from
// (reaching) v is either in v's closure or behind a node that is.
//
// Seed rows (fint(r) forward for every expandable r, rev(t) backward for every node t) sit
// in NODE BLOCKS: block v = `block` records (a power of two, 4..32: 64..512 bytes, aligned
// to its size) whose first record is a header {count, first record low, high, 0}; a row of
// at most block - 1 entries follows its header inside the block, so one request's seed row
// is one header read plus records on the same cache line(s); longer rows are kept whole in
// an overflow region and the header points there.
//
// Layout per direction d (0 forward, 1 backward): rec[d] = [core rows | closure rows | pad
// | node blocks | overflow rows].  Every record {node, deg, begin, pad}: the node's own
// expansion row in this array (closure or core row; 0/0 for a node with nothing to expand
// or outside the interior), pad flags below; unused block slots are {NONE, 0, 0, 0}.
#pragma once

#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

#include "ketogpu_internal.hpp"

namespace ketogpu {

// host threads of the index builders (KETOGPU_BUILD_THREADS; default at most 16: the GPU
// box's job quota, whatever nproc shows)
int build_threads();

// f(thread, begin, end) over [0, n) in chunks, on build_threads() threads
template <class F>
void parallel_chunks(uint64_t n, uint64_t chunk, F &&f) {
    const int T = build_threads();
    std::atomic<uint64_t> next{0};
    auto work = [&](int tid) {
        for (;;) {
            const uint64_t b = next.fetch_add(chunk);
            if (b >= n) return;
            f(tid, b, std::min(n, b + chunk));
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
}

struct CoreRec {
    uint32_t node, deg, begin, pad;
};
constexpr uint32_t kRecTerminal = 0x80000000u;  // an entry of a closure row: visited, never pending
constexpr uint32_t kRecClosure = 0x40000000u;   // deg/begin name the node's closure row

struct CoreIndex {
    std::vector<CoreRec> rec[2];
    uint64_t block_base[2] = {0, 0};       // record index of node 0's block
    uint32_t block_log[2] = {0, 0};        // log2 of the records per block
    uint64_t overflow_rows[2] = {0, 0};    // seed rows longer than a block holds
    uint64_t closure_nodes[2] = {0, 0};    // interior nodes with a closure row
    uint64_t closure_entries[2] = {0, 0};  // records in closure rows
    // per interior node: its closure row's length and first record (NONE: none)
    std::vector<uint32_t> clo_len[2], clo_beg[2];
    double build_ms = 0;
};

// cap[d]: the largest closure row kept in direction d (0: no closure rows).  block[d]:
// records per node block (a power of two in 4..32), 0 = chosen from the row lengths (the
// smallest block holding at least 95% of the non-empty seed rows).  Throws
// Error(KETOGPU_EINVAL) when the core and closure rows pass 2^32 records (32-bit begins).
// max_bytes: Error(KETOGPU_ENOMEM) when both directions' records pass it (0: no limit),
// before the record arrays are allocated.
void build_core_index(const Snapshot &s, const uint32_t cap[2], const uint32_t block[2], CoreIndex &out,
                      uint64_t max_bytes = 0);

}  // namespace ketogpu
