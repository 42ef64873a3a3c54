// part_round.cpp — the partitioned round, driven natively (include/ketogpu.h "whole rounds").
//
// One protocol for every communicator and every kind of steps (part_round.hpp): a round of
// up to 64 * round_words requests is
//
//   begin -> { emit -> [all-gather counts + status] -> stop when no rank sends anything
//                   -> [all-to-all records] -> apply -> expand }
//         -> pull_emit -> [all-gather counts + status] -> [all-to-all] -> pull_answer
//         -> end -> [all-gather hit bits + status] -> OR
//
// Two collectives per BFS level.  The counts all-gather carries every rank's step status,
// so a step that fails on one rank fails the round on all of them in the same collective
// (no rank waits in a collective its peers never enter), and the full count matrix, so
// every rank knows every receive size (the all-to-all needs no second count exchange) and
// the level where nothing moves anywhere ends the closure: frontier entries always have
// rows, so a non-empty frontier anywhere sends records (R2: no depth cutoff).
//
// This replaces keto_amd/partition.py's torch.distributed loop (three collectives and a
// Python round trip per level) so the Go host drives a partitioned PermissionEngine
// through one C call per batch (internal/driver/registry_default.go:158-163).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "part_round.hpp"

using namespace ketogpu;

namespace {

#define RHIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

// host steps from the caller's vtable (test hook)
struct VtableSteps : Steps {
    ketogpu_part_steps v{};
    std::string err;
    int rc(int code, const char *what) {
        if (code) err = std::string("partition steps: ") + what + " returned " + std::to_string(code);
        return code;
    }
    uint64_t round_words() override { return v.round_words; }
    uint64_t record_capacity() override { return 1 << 20; }
    int begin(const uint32_t *r, const uint32_t *t, uint64_t n, int dir) override {
        return rc(v.begin(v.ctx, r, t, n, dir), "begin");
    }
    int emit(int pull, ketogpu_record *send, uint64_t cap, uint64_t *counts) override {
        return rc(v.emit(v.ctx, pull, send, cap, counts), pull ? "pull_emit" : "emit");
    }
    int apply(const ketogpu_record *recv, uint64_t n, uint64_t *frontier) override {
        return rc(v.apply(v.ctx, recv, n, frontier), "apply");
    }
    int expand() override { return rc(v.expand(v.ctx), "expand"); }
    int pull_answer(const ketogpu_record *recv, uint64_t n) override {
        return rc(v.pull_answer(v.ctx, recv, n), "pull_answer");
    }
    int end(uint64_t *bits) override { return rc(v.end(v.ctx, bits), "end"); }
    int abort() override { return rc(v.abort(v.ctx), "abort"); }
    std::string error() override { return err; }
};

using Clock = std::chrono::steady_clock;

}  // namespace

struct ketogpu_part_engine {
    std::unique_ptr<Steps> steps;
    Comm *comm = nullptr;  // borrowed; null: one rank, no exchange
    int rank = 0, world = 1;
    int mode = KETOGPU_PART_AUTO, dir = KETOGPU_PART_AUTO;
    uint64_t per[2] = {~0ull, ~0ull};  // requests per round after overflow retries, per direction
    uint64_t top = 64;                 // requests one round holds (min over ranks)
    uint64_t cap = 0;                  // records per exchange buffer (min over ranks)
    // record buffers in the steps' memory, and staging in host memory when the steps are
    // device memory and the transport is host memory
    ketogpu_record *send = nullptr, *recv = nullptr;
    ketogpu_record *hsend = nullptr, *hrecv = nullptr;
    bool stage = false;
    // small collective buffers in the communicator's memory (RCCL: device)
    uint64_t *small_d = nullptr;
    uint64_t small_cap = 0;
    std::vector<uint64_t> mat, mine;
    std::mutex mu;
    ketogpu_part_engine_stats st{};

    ~ketogpu_part_engine() {
        if (steps && steps->device) {
            (void)hipSetDevice(steps->dev);
            if (steps->stream) (void)hipStreamSynchronize(steps->stream);
            for (void *p : {(void *)send, (void *)recv, (void *)small_d})
                if (p) (void)hipFree(p);
            for (void *p : {(void *)hsend, (void *)hrecv})
                if (p) (void)hipHostFree(p);
        } else {
            free(send);
            free(recv);
        }
    }

    hipStream_t stream() const { return steps->stream; }

    // every rank's n u64 values -> mat (world * n, rank order); host arrays
    void gather(const uint64_t *v, size_t n) {
        mat.assign(n * world, 0);
        if (!comm) {
            std::copy(v, v + n, mat.begin());
            return;
        }
        const auto t0 = Clock::now();
        if (comm->device) {
            const uint64_t need = n * (world + 1);
            if (need > small_cap) {
                if (small_d) (void)hipFree(small_d);
                small_d = nullptr;
                small_cap = std::max<uint64_t>(need, 1024);
                RHIP(hipMalloc(&small_d, small_cap * 8));
            }
            RHIP(hipMemcpyAsync(small_d, v, n * 8, hipMemcpyHostToDevice, stream()));
            comm->allgather(small_d, small_d + n, n * 8, stream());
            RHIP(hipMemcpyAsync(mat.data(), small_d + n, n * world * 8, hipMemcpyDeviceToHost, stream()));
            RHIP(hipStreamSynchronize(stream()));
        } else {
            comm->allgather(v, mat.data(), n * 8, stream());
        }
        st.collectives++;
        st.exchange_ms += std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    }

    // The level's collectives.  counts: this rank's records per destination (ignored when
    // code != 0).  -> agreed status (max over ranks), *n_in records received into rbuf(),
    // *moved = records sent by all ranks together
    int exchange(int code, const uint64_t *counts, uint64_t *n_in, uint64_t *moved) {
        *n_in = *moved = 0;
        const size_t W1 = (size_t)world + 1;
        if (!comm) {  // one rank: the records stay where the steps wrote them
            if (code) return code;
            *n_in = *moved = counts[0];
            if (counts[0] > cap) return KETOGPU_ENOMEM;
            st.records_sent += counts[0];
            st.records_received += counts[0];
            return KETOGPU_OK;
        }
        mine.assign(W1, 0);
        if (!code) std::copy(counts, counts + world, mine.begin());
        mine[world] = (uint64_t)code;
        gather(mine.data(), W1);
        int agreed = 0;
        uint64_t total = 0, most_in = 0;
        for (int r = 0; r < world; r++) agreed = std::max(agreed, (int)mat[r * W1 + world]);
        if (agreed) return agreed;
        for (int d = 0; d < world; d++) {
            uint64_t in = 0;
            for (int r = 0; r < world; r++) in += mat[r * W1 + d];
            total += in;
            most_in = std::max(most_in, in);
        }
        *moved = total;
        if (!total) return KETOGPU_OK;
        // every rank sees the whole matrix, so a receive overflow anywhere is known everywhere
        if (most_in > cap) return KETOGPU_ENOMEM;
        std::vector<uint64_t> sb(world), rb(world);
        uint64_t ns = 0, nr = 0;
        for (int p = 0; p < world; p++) {
            sb[p] = 16 * mat[rank * W1 + p];
            rb[p] = 16 * mat[p * W1 + rank];
            ns += sb[p];
            nr += rb[p];
        }
        const auto t0 = Clock::now();
        if (stage) {  // device steps, host transport
            RHIP(hipMemcpyAsync(hsend, send, ns, hipMemcpyDeviceToHost, stream()));
            RHIP(hipStreamSynchronize(stream()));
            comm->alltoallv(hsend, sb.data(), hrecv, rb.data(), stream());
            RHIP(hipMemcpyAsync(recv, hrecv, nr, hipMemcpyHostToDevice, stream()));
            RHIP(hipStreamSynchronize(stream()));
        } else {
            // RCCL on the steps' stream: ordered after the emit, before the apply
            comm->alltoallv(send, sb.data(), recv, rb.data(), stream());
        }
        st.collectives++;
        st.exchange_ms += std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
        *n_in = nr / 16;
        st.records_sent += ns / 16;
        st.records_received += nr / 16;
        return KETOGPU_OK;
    }
    const ketogpu_record *rbuf() const { return comm ? recv : send; }

    // a failed round: every rank aborts; ENOMEM is returned (retry smaller), anything else
    // raised with this rank's message when the failure was its own
    int fail(int code, int local) {
        const std::string why = local == code ? steps->error() : std::string();
        steps->abort();
        if (code == KETOGPU_ENOMEM) return code;
        throw Error(code, why.empty() ? "partition: a step failed on another rank" : why);
    }

    // one round; bits: ceil(n/64) words.  0, or ENOMEM after every rank aborted it
    int round(const uint32_t *r, const uint32_t *t, uint64_t n, int d, uint64_t *bits) {
        st.rounds++;
        uint64_t counts[64], n_in = 0, moved = 0, frontier = 0;
        int local = steps->begin(r, t, n, d);  // reported with the first emit
        for (;;) {
            if (!local) local = steps->emit(0, send, cap, counts);
            const int code = exchange(local, counts, &n_in, &moved);
            if (code) return fail(code, local);
            if (!moved) break;  // no rank has a frontier left: the closures are complete
            st.levels++;
            local = steps->apply(rbuf(), n_in, &frontier);
            if (!local && frontier) local = steps->expand();
        }
        local = steps->emit(1, send, cap, counts);
        int code = exchange(local, counts, &n_in, &moved);
        if (code) return fail(code, local);
        local = steps->pull_answer(rbuf(), n_in);
        const uint64_t words = (n + 63) / 64;
        std::fill(bits, bits + words, 0);
        if (!local) local = steps->end(bits);
        if (comm) {  // the answer is the OR of the ranks' hit bits; the last word is the status
            std::vector<uint64_t> v(bits, bits + words);
            v.push_back((uint64_t)local);
            gather(v.data(), words + 1);
            code = 0;
            for (int k = 0; k < world; k++) code = std::max(code, (int)mat[k * (words + 1) + words]);
            if (!code)
                for (int k = 0; k < world; k++)
                    for (uint64_t w = 0; w < words; w++) bits[w] |= mat[k * (words + 1) + w];
        } else {
            code = local;
        }
        if (code) return fail(code, local);
        return KETOGPU_OK;
    }

    void shrink(int d, uint64_t m) {
        if (m <= 64) throw Error(KETOGPU_ENOMEM, "partition buffers overflow for a single 64-request word");
        per[d] = std::max<uint64_t>(64, (m / 2) / 64 * 64);
        st.retries++;
    }

    uint64_t max_over_ranks(uint64_t v) {
        gather(&v, 1);
        uint64_t m = 0;
        for (int k = 0; k < world; k++) m = std::max(m, mat[k]);
        return m;
    }

    void check_ids(const uint32_t *roots, const uint32_t *targets, uint64_t n, uint64_t *out) {
        if (steps->device) RHIP(hipSetDevice(steps->dev));
        std::vector<uint64_t> a, b;
        uint64_t i = 0;
        while (i < n) {
            if (dir == KETOGPU_PART_AUTO) {
                // both directions run the SAME first round (equal work), timed, max over
                // ranks so every rank decides alike; the faster is kept
                const uint64_t m = std::min({top, per[0], per[1], n - i});
                a.assign((m + 63) / 64, 0);
                b.assign((m + 63) / 64, 0);
                uint64_t ns[2];
                int rc[2];
                for (int d = 0; d < 2; d++) {
                    const auto t0 = Clock::now();
                    rc[d] = round(roots + i, targets + i, m, d, d ? b.data() : a.data());
                    ns[d] = max_over_ranks(
                        (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count() /
                        std::max<uint64_t>(m, 1));
                }
                if (rc[0] || rc[1]) {  // ENOMEM, agreed by every rank
                    for (int d = 0; d < 2; d++) shrink(d, m);
                    continue;
                }
                if (a != b) throw Error(KETOGPU_EDEVICE, "partition: forward and backward rounds disagree");
                st.trial_ns[0] = ns[0];
                st.trial_ns[1] = ns[1];
                dir = ns[1] < ns[0] ? KETOGPU_PART_BACKWARD : KETOGPU_PART_FORWARD;
                st.direction = dir;
                std::copy(a.begin(), a.end(), out + i / 64);
                i += m;
                continue;
            }
            const uint64_t m = std::min({top, per[dir], n - i});
            a.assign((m + 63) / 64, 0);
            if (round(roots + i, targets + i, m, dir, a.data())) {
                shrink(dir, m);  // a round size that overflowed stays halved for later calls
                continue;
            }
            std::copy(a.begin(), a.end(), out + i / 64);  // i is a multiple of 64 (m is, but the last)
            i += m;
        }
    }

    void init(std::unique_ptr<Steps> s, ketogpu_comm *c, const ketogpu_part_engine_opts *o) {
        steps = std::move(s);
        comm = c ? c->c.get() : nullptr;
        rank = comm ? comm->rank : 0;
        world = comm ? comm->world : 1;
        mode = dir = o ? o->direction : KETOGPU_PART_AUTO;
        if (mode != KETOGPU_PART_AUTO && mode != KETOGPU_PART_FORWARD && mode != KETOGPU_PART_BACKWARD)
            throw Error(KETOGPU_EINVAL, "partition engine: direction must be FORWARD, BACKWARD or AUTO");
        st.direction = dir;
        if (comm && comm->device && (!steps->device || comm->dev != steps->dev))
            throw Error(KETOGPU_EINVAL, "partition engine: an RCCL communicator needs device steps on its device");
        stage = comm && steps->device && !comm->device;
        // every rank uses the same round size and buffer capacity (one collective, here)
        uint64_t want[2] = {steps->round_words() * 64, o && o->record_capacity ? o->record_capacity
                                                                               : steps->record_capacity()};
        if (steps->device) RHIP(hipSetDevice(steps->dev));
        uint64_t agreed[2] = {want[0], want[1]};
        if (comm) {
            gather(want, 2);
            for (int k = 0; k < world; k++) {
                agreed[0] = std::min(agreed[0], mat[2 * k]);
                agreed[1] = std::min(agreed[1], mat[2 * k + 1]);
            }
        }
        top = std::max<uint64_t>(64, agreed[0] / 64 * 64);
        cap = std::max<uint64_t>(agreed[1], 1);
        // the steps must write their records into `send` when an exchange reads them
        steps->set_exchange(comm != nullptr);
        if (steps->device) {
            RHIP(hipMalloc(&send, cap * sizeof(ketogpu_record)));
            if (comm) RHIP(hipMalloc(&recv, cap * sizeof(ketogpu_record)));
            if (stage) {
                RHIP(hipHostMalloc((void **)&hsend, cap * sizeof(ketogpu_record), hipHostMallocDefault));
                RHIP(hipHostMalloc((void **)&hrecv, cap * sizeof(ketogpu_record), hipHostMallocDefault));
            }
        } else {
            send = (ketogpu_record *)malloc(cap * sizeof(ketogpu_record));
            recv = (ketogpu_record *)malloc(cap * sizeof(ketogpu_record));
            if (!send || !recv) throw std::bad_alloc();
        }
    }
};

#define RAPI_BEGIN try {
#define RAPI_END                                                                                       \
    }                                                                                                  \
    catch (const Error &e) {                                                                           \
        set_last_error(e.what());                                                                      \
        return e.code;                                                                                 \
    }                                                                                                  \
    catch (const std::bad_alloc &) {                                                                   \
        set_last_error("out of host memory");                                                          \
        return KETOGPU_ENOMEM;                                                                         \
    }                                                                                                  \
    return KETOGPU_OK;

extern "C" {

int ketogpu_part_engine_new(ketogpu_part *p, ketogpu_comm *c, const ketogpu_part_engine_opts *opts,
                            ketogpu_part_engine **out) {
    RAPI_BEGIN
    if (!p || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto e = std::make_unique<ketogpu_part_engine>();
    e->init(device_steps(p), c, opts);
    *out = e.release();
    RAPI_END
}

int ketogpu_part_engine_new_steps(const ketogpu_part_steps *steps, ketogpu_comm *c,
                                  const ketogpu_part_engine_opts *opts, ketogpu_part_engine **out) {
    RAPI_BEGIN
    if (!steps || !out || !steps->begin || !steps->emit || !steps->apply || !steps->expand || !steps->pull_answer ||
        !steps->end || !steps->abort || !steps->round_words)
        throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    auto s = std::make_unique<VtableSteps>();
    s->v = *steps;
    auto e = std::make_unique<ketogpu_part_engine>();
    e->init(std::move(s), c, opts);
    *out = e.release();
    RAPI_END
}

void ketogpu_part_engine_free(ketogpu_part_engine *e) { delete e; }

int ketogpu_part_check_ids(ketogpu_part_engine *e, const uint32_t *roots, const uint32_t *targets, size_t n,
                           uint64_t *allowed_bits) {
    RAPI_BEGIN
    if (!e || (n && (!roots || !targets || !allowed_bits))) throw Error(KETOGPU_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    e->check_ids(roots, targets, n, allowed_bits);
    RAPI_END
}

int ketogpu_part_engine_stats_get(const ketogpu_part_engine *e, ketogpu_part_engine_stats *out) {
    if (!e || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    *out = e->st;
    return KETOGPU_OK;
}

int ketogpu_part_resolve_batch(const ketogpu_shard *s, ketogpu_comm *c, const ketogpu_request_batch *reqs,
                               uint32_t *roots, uint32_t *targets, int32_t *status) {
    RAPI_BEGIN
    if (!s || !reqs || (reqs->n && (!roots || !targets || !status))) throw Error(KETOGPU_EINVAL, "null argument");
    // every rank resolves locally (no early return: a failure here still joins the
    // collectives below, its code travels in the status lane)
    int rc = ketogpu_shard_resolve_batch(s, reqs, roots, targets, status);
    const std::string why = rc ? std::string(ketogpu_last_error()) : std::string();
    Comm *comm = c ? c->c.get() : nullptr;
    const uint64_t n = reqs->n;
    if (comm && comm->world > 1) {
        // the owners' ids win: MIN with "not owned" mapped above every id and "none"
        std::vector<uint32_t> v(2 * n + 1), w(n + 1);
        for (uint64_t i = 0; i < n; i++) {
            for (int k = 0; k < 2; k++) {
                const uint32_t x = rc ? KETOGPU_NODE_NOT_OWNED : (k ? targets[i] : roots[i]);
                v[k * n + i] = x == KETOGPU_NODE_NOT_OWNED ? 0xFFFFFFFFu : x == KETOGPU_NODE_NONE ? 0xFFFFFFFEu : x;
            }
            w[i] = rc ? 0u : (uint32_t)status[i];
        }
        v[2 * n] = 0;
        w[n] = (uint32_t)rc;
        auto reduce = [&](std::vector<uint32_t> &x, int op) {
            if (comm->device) {
                RHIP(hipSetDevice(comm->dev));
                uint32_t *d = nullptr;
                RHIP(hipMalloc(&d, x.size() * 4));
                try {
                    RHIP(hipMemcpy(d, x.data(), x.size() * 4, hipMemcpyHostToDevice));
                    comm->allreduce_u32(d, x.size(), op, nullptr);
                    comm->wait(nullptr);
                    RHIP(hipMemcpy(x.data(), d, x.size() * 4, hipMemcpyDeviceToHost));
                } catch (...) {
                    (void)hipFree(d);
                    throw;
                }
                (void)hipFree(d);
            } else {
                comm->allreduce_u32(x.data(), x.size(), op, nullptr);
            }
        };
        reduce(v, KETOGPU_REDUCE_MIN);
        reduce(w, KETOGPU_REDUCE_MAX);
        if (w[n]) throw Error((int)w[n], rc ? why : "partition: request resolution failed on another rank");
        for (uint64_t i = 0; i < n; i++) {
            roots[i] = v[i] >= 0xFFFFFFFEu ? KETOGPU_NODE_NONE : v[i];
            targets[i] = v[n + i] >= 0xFFFFFFFEu ? KETOGPU_NODE_NONE : v[n + i];
            status[i] = (int32_t)w[i];
        }
    } else if (rc) {
        throw Error(rc, why);
    } else {
        for (uint64_t i = 0; i < n; i++) {  // one rank owns everything
            if (roots[i] == KETOGPU_NODE_NOT_OWNED) roots[i] = KETOGPU_NODE_NONE;
            if (targets[i] == KETOGPU_NODE_NOT_OWNED) targets[i] = KETOGPU_NODE_NONE;
        }
    }
    RAPI_END
}

}  // extern "C"

namespace {
// a communicator of one rank (ketogpu_shard_exchange without one): collectives copy
struct SelfComm : Comm {
    void allgather(const void *send, void *recv, uint64_t bytes, hipStream_t) override { memcpy(recv, send, bytes); }
    void alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *, hipStream_t) override {
        memcpy(recv, send, sb[0]);
    }
    void allreduce_u32(uint32_t *, uint64_t, int, hipStream_t) override {}
    void wait(hipStream_t) override {}
};
}  // namespace

// ------------------------------------------------ the loader's id exchange
// Collectives on host arrays over any communicator (part_round.hpp HostColl; RCCL:
// staged through device memory).
namespace ketogpu {
HostColl::~HostColl() {
    if (dbuf) (void)hipFree(dbuf);
}

char *HostColl::dev(uint64_t bytes) {
    if (bytes > dcap) {
        if (dbuf) (void)hipFree(dbuf);
        dbuf = nullptr;
        dcap = std::max<uint64_t>(bytes, 4096);
        RHIP(hipMalloc(&dbuf, dcap));
    }
    return (char *)dbuf;
}

void HostColl::allgather(const void *send, void *recv, uint64_t bytes) {
    if (!c->device) return c->allgather(send, recv, bytes, nullptr);
    RHIP(hipSetDevice(c->dev));
    char *d = dev(bytes * (c->world + 1));
    RHIP(hipMemcpy(d, send, bytes, hipMemcpyHostToDevice));
    c->allgather(d, d + bytes, bytes, nullptr);
    c->wait(nullptr);
    RHIP(hipMemcpy(recv, d + bytes, bytes * c->world, hipMemcpyDeviceToHost));
}

const std::vector<uint64_t> &HostColl::gather(const std::vector<uint64_t> &v) {
    mat.assign(v.size() * c->world, 0);
    allgather(v.data(), mat.data(), v.size() * 8);
    return mat;
}

int HostColl::agree(int rc) {
    gather({(uint64_t)rc});
    int m = 0;
    for (uint64_t x : mat) m = std::max(m, (int)x);
    return m;
}

std::vector<char> HostColl::alltoallv(const void *send, const std::vector<uint64_t> &counts, uint64_t unit,
                                      std::vector<uint64_t> *rcounts) {
    const int W = c->world, me = c->rank;
    gather(counts);
    std::vector<uint64_t> sb(W), rb(W);
    uint64_t ns = 0, nr = 0;
    for (int p = 0; p < W; p++) {
        sb[p] = counts[p] * unit;
        rb[p] = mat[(size_t)p * W + me] * unit;
        ns += sb[p];
        nr += rb[p];
    }
    if (rcounts) {
        rcounts->resize(W);
        for (int p = 0; p < W; p++) (*rcounts)[p] = rb[p] / unit;
    }
    std::vector<char> out(nr);
    if (!c->device) {
        c->alltoallv(send, sb.data(), out.data(), rb.data(), nullptr);
        return out;
    }
    RHIP(hipSetDevice(c->dev));
    char *d = dev(ns + nr);
    if (ns) RHIP(hipMemcpy(d, send, ns, hipMemcpyHostToDevice));
    c->alltoallv(d, sb.data(), d + ns, rb.data(), nullptr);
    c->wait(nullptr);
    if (nr) RHIP(hipMemcpy(out.data(), d + ns, nr, hipMemcpyDeviceToHost));
    return out;
}

std::vector<char> HostColl::allgatherv(const void *send, uint64_t bytes, std::vector<uint64_t> *sizes) {
    const int W = c->world;
    std::vector<uint64_t> counts(W, bytes);
    std::vector<uint64_t> rc;
    // the same bytes to every rank: an all-to-all whose every send part is the whole buffer
    std::vector<char> rep((size_t)bytes * W);
    for (int p = 0; p < W; p++)
        if (bytes) memcpy(rep.data() + (size_t)p * bytes, send, bytes);
    std::vector<char> out = alltoallv(rep.data(), counts, 1, &rc);
    if (sizes) *sizes = rc;
    return out;
}
}  // namespace ketogpu

extern "C" {

int ketogpu_shard_exchange(ketogpu_shard *s, ketogpu_comm *comm) {
    RAPI_BEGIN
    if (!s) throw Error(KETOGPU_EINVAL, "null argument");
    ketogpu_comm one{};
    if (!comm) {  // a single rank: a one-member transport that copies
        auto cc = std::make_unique<SelfComm>();
        one.c = std::move(cc);
        comm = &one;
    }
    HostColl hc{comm->c.get()};
    const int W = hc.c->world;
    std::string why;
    auto step = [&](int rc) {  // a local step's status, agreed by every rank
        if (rc) why = ketogpu_last_error();
        const int a = hc.agree(rc);
        if (a) throw Error(a, rc == a ? why : std::string("shard loading failed on another rank"));
    };
    // 1. per-class node counts -> the global id layout
    std::vector<uint64_t> cnt(3, 0);
    step(ketogpu_shard_counts(s, cnt.data()));
    std::vector<uint64_t> all = hc.gather(cnt);
    step(ketogpu_shard_set_layout(s, all.data()));
    // 2. node ids: hashes to their owners, ids back in the same order
    const uint64_t nq = ketogpu_shard_query_count(s);
    std::vector<uint64_t> q(std::max<uint64_t>(nq, 1)), qc(W);
    step(ketogpu_shard_queries(s, q.data(), nq, qc.data()));
    std::vector<uint64_t> rc;
    std::vector<char> got = hc.alltoallv(q.data(), qc, 8, &rc);
    const uint64_t nr = got.size() / 8;
    std::vector<uint32_t> ids(std::max<uint64_t>(nr, 1));
    step(ketogpu_shard_answer(s, (const uint64_t *)got.data(), nr, ids.data()));
    std::vector<char> back = hc.alltoallv(ids.data(), rc, 4, nullptr);
    if (back.size() != nq * 4) throw Error(KETOGPU_EDEVICE, "shard exchange: answers do not match the queries");
    step(ketogpu_shard_apply(s, nq ? (const uint32_t *)back.data() : nullptr, nq));
    // 3. R4: shared Subject.String() keys, counted by the key hashes' owners
    const uint64_t nc = ketogpu_shard_claim_count(s);
    std::vector<uint64_t> pairs(std::max<uint64_t>(2 * nc, 2)), pc(W);
    step(ketogpu_shard_claims(s, pairs.data(), nc, pc.data()));
    std::vector<char> cl = hc.alltoallv(pairs.data(), pc, 16, nullptr);
    uint64_t amb = 0;
    step(ketogpu_shard_check_claims(s, (const uint64_t *)cl.data(), cl.size() / 16, &amb));
    uint64_t total = 0;
    for (uint64_t x : hc.gather({amb})) total += x;
    if (total)
        throw Error(KETOGPU_EINVAL, "partitioned loader: " + std::to_string(total) +
                                        " Subject.String() keys are shared by two nodes (R4); load this network "
                                        "with the whole-graph snapshot");
    RAPI_END
}

}  // extern "C"
