// comm.cpp — communicators of the partitioned mode (include/ketogpu.h "whole rounds").
//
// RcclComm: RCCL over xGMI, one process per GPU (SURVEY.md 8(e) "Partitioned"; the
// reference itself has no collectives: it scales out by stateless processes on one DB,
// internal/driver/daemon.go:87-159).  librccl is opened at the first communicator, not
// linked: the library loads on hosts without it (the CPU test suite), and in a process
// that already holds RCCL (torch) dlopen returns that same copy (same SONAME).  Records
// move from device memory on the caller's stream: grouped ncclSend/ncclRecv per peer
// (a per-link exchange: xGMI is point to point, one ~153 GB/s link per peer pair in an
// 8-GPU node) and small ncclAllGather / ncclAllReduce for counts and answers.
//
// CallbackComm: the caller's transport vtable over host memory (a Go transport; the CPU
// tests' torch.distributed gloo).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "part_round.hpp"

using namespace ketogpu;

namespace {

#define CHIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t _e = (x);                                                                           \
        if (_e != hipSuccess) throw Error(KETOGPU_EDEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

// the RCCL entry points this file uses, resolved once
struct RcclApi {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    std::string err;
};

const RcclApi &rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
        if (!h) {
            const char *e = dlerror();
            api.err = std::string("librccl: ") + (e ? e : "not found");
            return;
        }
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && api.err.empty()) api.err = std::string("librccl: no symbol ") + name;
        };
        sym(api.GetUniqueId, "ncclGetUniqueId");
        sym(api.CommInitRank, "ncclCommInitRank");
        sym(api.CommDestroy, "ncclCommDestroy");
        sym(api.GetErrorString, "ncclGetErrorString");
        sym(api.GroupStart, "ncclGroupStart");
        sym(api.GroupEnd, "ncclGroupEnd");
        sym(api.Send, "ncclSend");
        sym(api.Recv, "ncclRecv");
        sym(api.AllGather, "ncclAllGather");
        sym(api.AllReduce, "ncclAllReduce");
    });
    if (!api.err.empty()) throw Error(KETOGPU_EDEVICE, api.err);
    return api;
}

void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) {
        const RcclApi &a = rccl();
        throw Error(KETOGPU_EDEVICE, std::string(what) + ": " + (a.GetErrorString ? a.GetErrorString(r) : "rccl error"));
    }
}

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) {
            (void)hipSetDevice(dev);
            (void)hipDeviceSynchronize();  // no operation of this communicator in flight
            rccl().CommDestroy(comm);
        }
    }
    void allgather(const void *send, void *recv, uint64_t bytes, hipStream_t s) override {
        CHIP(hipSetDevice(dev));
        nccl_check(rccl().AllGather(send, recv, bytes, ncclUint8, comm, s), "ncclAllGather");
        n_allgather++;
    }
    void alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb, hipStream_t s) override {
        CHIP(hipSetDevice(dev));
        const RcclApi &a = rccl();
        uint64_t so = 0, ro = 0;
        for (int p = 0; p < rank; p++) so += sb[p], ro += rb[p];
        // the rank's own segment: a copy engine's DMA on the same stream (RCCL's self
        // send/receive runs as a kernel at ~1 TB/s); loop_self (tests): through RCCL
        if (sb[rank] != rb[rank]) throw Error(KETOGPU_EINVAL, "alltoallv: own segment sizes differ");
        if (sb[rank] && !loop_self)
            CHIP(hipMemcpyAsync((char *)recv + ro, (const char *)send + so, sb[rank], hipMemcpyDeviceToDevice, s));
        if (world == 1 && !loop_self) return;
        nccl_check(a.GroupStart(), "ncclGroupStart");
        so = ro = 0;
        for (int p = 0; p < world; p++) {
            // one send and one receive per peer in one group: RCCL runs them concurrently,
            // one xGMI link per peer pair
            const bool peer = p != rank || loop_self;
            if (peer && sb[p]) {
                nccl_check(a.Send((const char *)send + so, sb[p], ncclUint8, p, comm, s), "ncclSend");
                n_send++;
                bytes_sent += sb[p];
            }
            if (peer && rb[p]) {
                nccl_check(a.Recv((char *)recv + ro, rb[p], ncclUint8, p, comm, s), "ncclRecv");
                n_recv++;
            }
            so += sb[p];
            ro += rb[p];
        }
        nccl_check(a.GroupEnd(), "ncclGroupEnd");
    }
    void allreduce_u32(uint32_t *buf, uint64_t n, int op, hipStream_t s) override {
        CHIP(hipSetDevice(dev));
        nccl_check(rccl().AllReduce(buf, buf, n, ncclUint32, op == KETOGPU_REDUCE_MIN ? ncclMin : ncclMax, comm, s),
                   "ncclAllReduce");
        n_allreduce++;
    }
    void wait(hipStream_t s) override { CHIP(hipStreamSynchronize(s)); }
};

struct CallbackComm : Comm {
    ketogpu_transport t{};
    void fail(const char *what) {
        throw Error(KETOGPU_EDEVICE, std::string("transport ") + what + " failed on rank " + std::to_string(rank));
    }
    void allgather(const void *send, void *recv, uint64_t bytes, hipStream_t) override {
        if (t.allgather(t.ctx, send, recv, bytes)) fail("allgather");
    }
    void alltoallv(const void *send, const uint64_t *sb, void *recv, const uint64_t *rb, hipStream_t) override {
        if (t.alltoallv(t.ctx, send, sb, recv, rb)) fail("alltoallv");
    }
    void allreduce_u32(uint32_t *buf, uint64_t n, int op, hipStream_t) override {
        if (t.allreduce_u32(t.ctx, buf, n, op)) fail("allreduce_u32");
    }
    void wait(hipStream_t) override {}
};

#define CAPI_BEGIN try {
#define CAPI_END                                                                                       \
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

}  // namespace

extern "C" {

int ketogpu_comm_unique_id(uint8_t id[KETOGPU_COMM_ID_BYTES]) {
    CAPI_BEGIN
    if (!id) throw Error(KETOGPU_EINVAL, "null argument");
    static_assert(sizeof(ncclUniqueId) == KETOGPU_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    nccl_check(rccl().GetUniqueId(&u), "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
    CAPI_END
}

int ketogpu_comm_new(const uint8_t id[KETOGPU_COMM_ID_BYTES], int32_t rank, int32_t world, int32_t device,
                     ketogpu_comm **out) {
    CAPI_BEGIN
    if (!id || !out) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    if (world < 1 || world > 64 || rank < 0 || rank >= world)
        throw Error(KETOGPU_EINVAL, "comm: need 0 <= rank < world <= 64");
    int ndev = 0;
    CHIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw Error(KETOGPU_EDEVICE, "no such HIP device");
    CHIP(hipSetDevice(device));
    auto c = std::make_unique<RcclComm>();
    c->rank = rank;
    c->world = world;
    c->device = true;
    c->dev = device;
    c->loop_self = getenv("KETOGPU_TEST_RCCL_SELF") != nullptr;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    nccl_check(rccl().CommInitRank(&c->comm, world, u, rank), "ncclCommInitRank");
    auto h = std::make_unique<ketogpu_comm>();
    h->c = std::move(c);
    *out = h.release();
    CAPI_END
}

int ketogpu_comm_from_transport(const ketogpu_transport *t, ketogpu_comm **out) {
    CAPI_BEGIN
    if (!t || !out || !t->allgather || !t->alltoallv || !t->allreduce_u32) throw Error(KETOGPU_EINVAL, "null argument");
    *out = nullptr;
    if (t->world < 1 || t->world > 64 || t->rank < 0 || t->rank >= t->world)
        throw Error(KETOGPU_EINVAL, "transport: need 0 <= rank < world <= 64");
    auto c = std::make_unique<CallbackComm>();
    c->t = *t;
    c->rank = t->rank;
    c->world = t->world;
    auto h = std::make_unique<ketogpu_comm>();
    h->c = std::move(c);
    *out = h.release();
    CAPI_END
}

int ketogpu_comm_stats_get(const ketogpu_comm *c, ketogpu_comm_stats *out) {
    if (!c || !out) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    const Comm &m = *c->c;
    out->rccl = m.device ? 1 : 0;
    out->loop_self = m.loop_self ? 1 : 0;
    out->sends = m.n_send;
    out->recvs = m.n_recv;
    out->allgathers = m.n_allgather;
    out->allreduces = m.n_allreduce;
    out->bytes_sent = m.bytes_sent;
    return KETOGPU_OK;
}

void ketogpu_comm_free(ketogpu_comm *c) { delete c; }
int ketogpu_comm_rank(const ketogpu_comm *c) { return c ? c->c->rank : 0; }
int ketogpu_comm_world(const ketogpu_comm *c) { return c ? c->c->world : 1; }

}  // extern "C"
