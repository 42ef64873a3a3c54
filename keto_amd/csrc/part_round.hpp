// part_round.hpp — the partitioned mode's exchange, behind the C ABI (internal).
//
// A partitioned check round (SURVEY.md 8(e) "Partitioned") is one rank's device steps
// (partition.hip) interleaved with collectives between ranks.  Both sides are interfaces
// here so the ONE protocol implementation (part_round.cpp) drives every combination:
//
//   Comm   how ranks exchange bytes: RCCL over xGMI (device memory, on the partition's
//          stream; comm.cpp, librccl loaded at first use) or a caller's transport vtable
//          (host memory: a Go transport, torch.distributed gloo in the CPU tests)
//   Steps  one rank's steps of a round: the HIP partition (device memory) or a caller's
//          steps vtable (host memory; the CPU tests' stand-in, tests/part_cpu.py)
//
// The driver stages records between the two memories when they differ.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ketogpu_internal.hpp"

namespace ketogpu {

struct Comm {
    int rank = 0, world = 1;
    bool device = false;  // buffers are device memory of `dev` (RCCL) or host memory
    int dev = -1;
    // KETOGPU_TEST_RCCL_SELF=1 when an RCCL communicator is made: even at world 1 every
    // collective goes through RCCL (the own segment of an all-to-all as a grouped
    // ncclSend/ncclRecv to the rank itself, the count gathers as ncclAllGather), so the
    // data path a multi-GPU run takes is executed on one GPU
    bool loop_self = false;
    // RCCL calls made (ketogpu_comm_stats_get)
    uint64_t n_send = 0, n_recv = 0, n_allgather = 0, n_allreduce = 0, bytes_sent = 0;
    virtual ~Comm() = default;
    // every rank's `bytes` bytes -> recv (world * bytes, in rank order)
    virtual void allgather(const void *send, void *recv, uint64_t bytes, hipStream_t s) = 0;
    // send grouped by destination rank (send_bytes[world]) -> recv grouped by source rank
    // (recv_bytes[world]); both sizes are known to the caller beforehand
    virtual void alltoallv(const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes,
                           hipStream_t s) = 0;
    // elementwise, in place: KETOGPU_REDUCE_MIN / _MAX
    virtual void allreduce_u32(uint32_t *buf, uint64_t n, int op, hipStream_t s) = 0;
    // after an operation on stream s: its output is readable by the host
    virtual void wait(hipStream_t s) = 0;
};

// One rank's steps of a round (the ketogpu_part_* sequence).  Return codes are KETOGPU_*;
// KETOGPU_ENOMEM means "buffers too small for this round" (every rank aborts and retries
// with fewer requests).  error() is the message of the last failing step.
struct Steps {
    bool device = false;  // record buffers are device memory of `dev`
    int dev = -1;
    hipStream_t stream = nullptr;  // where the steps run (device steps)
    virtual ~Steps() = default;
    virtual uint64_t round_words() = 0;
    virtual uint64_t record_capacity() = 0;  // records per exchange buffer the steps suggest
    virtual int begin(const uint32_t *roots, const uint32_t *targets, uint64_t n, int dir) = 0;
    // pull = 0: the BFS level's records; 1: the pull queries.  Grouped by destination.
    virtual int emit(int pull, ketogpu_record *send, uint64_t capacity, uint64_t *counts) = 0;
    virtual int apply(const ketogpu_record *recv, uint64_t n, uint64_t *frontier) = 0;
    virtual int expand() = 0;
    virtual int pull_answer(const ketogpu_record *recv, uint64_t n) = 0;
    virtual int end(uint64_t *bits) = 0;
    virtual int abort() = 0;
    // make the last emit's send buffer complete for readers on other streams
    virtual void sync() {}
    // records must really be written into `send` even at world 1 (an exchange reads them)
    virtual void set_exchange(bool) {}
    virtual std::string error() = 0;
};

// Collectives on host arrays over any communicator (RCCL: staged through device memory
// of the communicator's GPU); load-time exchanges, not the per-batch path.
struct HostColl {
    Comm *c;
    std::vector<uint64_t> mat;
    void *dbuf = nullptr;
    uint64_t dcap = 0;
    explicit HostColl(Comm *cc) : c(cc) {}
    HostColl(const HostColl &) = delete;
    ~HostColl();
    char *dev(uint64_t bytes);
    void allgather(const void *send, void *recv, uint64_t bytes);
    // every rank's u64 list of the same length -> mat[world][k]
    const std::vector<uint64_t> &gather(const std::vector<uint64_t> &v);
    // status agreement: the largest code of any rank (0 when every rank succeeded)
    int agree(int rc);
    // variable all-to-all of `unit`-byte items: counts[world] items per destination
    std::vector<char> alltoallv(const void *send, const std::vector<uint64_t> &counts, uint64_t unit,
                                std::vector<uint64_t> *rcounts);
    // every rank's `bytes` bytes (any length per rank) -> their concatenation in rank order
    std::vector<char> allgatherv(const void *send, uint64_t bytes, std::vector<uint64_t> *sizes);
};

// partition.hip: the HIP steps of a ketogpu_part
std::unique_ptr<Steps> device_steps(ketogpu_part *p);

}  // namespace ketogpu

struct ketogpu_comm {
    std::unique_ptr<ketogpu::Comm> c;
};
