// multi_engine.cpp — replicated multi-GPU check engine (BASELINE configs #2-#4 at 1/2/4/8
// GPUs; SURVEY.md 8(e) "Replicated").
//
// The reference scales out by running more stateless Keto processes against one
// database (internal/driver/daemon.go:87-159); inside one process there is exactly one
// PermissionEngine (internal/driver/registry_default.go:158-163).  The replacement keeps
// one engine per process and spreads each batch over the node's GPUs itself: every
// device holds the whole graph (it fits 288 GB of HBM many times over), a batch is split
// into contiguous ranges of whole 64-request words, one range per device, run
// concurrently from one persistent host thread per device, and the result words are
// written straight into the caller's bit array at the range's offset (concatenation is
// free).  No data-path collective: checks are independent units.
#include <algorithm>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ketogpu_internal.hpp"

using namespace ketogpu;

struct ketogpu_multi {
    std::vector<ketogpu_engine *> eng;
    std::vector<std::thread> workers;
    std::mutex mu;       // job state below
    std::condition_variable start_cv, done_cv;
    uint64_t gen = 0;    // job generation
    size_t pending = 0;  // workers still running the current job
    bool stop = false;
    // the current job
    const uint32_t *roots = nullptr, *targets = nullptr;
    size_t n = 0;
    uint64_t *allowed = nullptr, *flagged = nullptr;
    std::vector<int> rc;
    std::vector<std::string> err;
    std::mutex call_mu;  // one batch at a time (each engine serializes its own calls too)

    ~ketogpu_multi() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        start_cv.notify_all();
        for (auto &t : workers)
            if (t.joinable()) t.join();
        for (auto *e : eng) ketogpu_engine_free(e);
    }

    void worker(size_t i) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                start_cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
            }
            size_t b = 0, e = 0;
            ketogpu_multi_range(n, eng.size(), i, &b, &e);
            int r = KETOGPU_OK;
            std::string msg;
            if (e > b) {
                r = ketogpu_check_ids(eng[i], roots + b, targets + b, e - b, allowed + b / 64,
                                      flagged ? flagged + b / 64 : nullptr);
                if (r) msg = ketogpu_last_error();  // thread-local: read on this thread
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                rc[i] = r;
                err[i] = std::move(msg);
                if (--pending == 0) done_cv.notify_all();
            }
        }
    }
};

extern "C" {

void ketogpu_multi_range(size_t n, size_t parts, size_t i, size_t *begin, size_t *end) {
    if (!begin || !end) return;
    *begin = *end = 0;
    if (!parts || i >= parts) return;
    const size_t words = (n + 63) / 64, q = words / parts, r = words % parts;
    const size_t w0 = i * q + std::min(i, r), w1 = w0 + q + (i < r ? 1 : 0);
    *begin = std::min(n, w0 * 64);
    *end = std::min(n, w1 * 64);
}

int ketogpu_multi_new(const ketogpu_snapshot *s, const int32_t *devices, size_t num_devices,
                      const ketogpu_engine_opts *opts, ketogpu_multi **out) {
    try {
        if (!s || !devices || !num_devices || !out) throw Error(KETOGPU_EINVAL, "null argument");
        *out = nullptr;
        for (size_t i = 0; i < num_devices; i++)
            for (size_t j = 0; j < i; j++)
                if (devices[i] == devices[j]) throw Error(KETOGPU_EINVAL, "a device is listed twice");
        auto m = std::make_unique<ketogpu_multi>();
        const size_t nd = num_devices;
        m->eng.assign(nd, nullptr);
        m->rc.assign(nd, KETOGPU_OK);
        m->err.assign(nd, std::string());
        // the engines upload the graph (and build their hub indexes) concurrently
        std::vector<std::thread> init;
        for (size_t i = 0; i < nd; i++)
            init.emplace_back([&, i] {
                ketogpu_engine_opts o = opts ? *opts : ketogpu_engine_opts{};
                o.device = devices[i];
                m->rc[i] = ketogpu_engine_new(s, &o, &m->eng[i]);
                if (m->rc[i]) m->err[i] = ketogpu_last_error();
            });
        for (auto &t : init) t.join();
        for (size_t i = 0; i < nd; i++)
            if (m->rc[i]) throw Error(m->rc[i], "device " + std::to_string(devices[i]) + ": " + m->err[i]);
        for (size_t i = 0; i < nd; i++) m->workers.emplace_back([p = m.get(), i] { p->worker(i); });
        *out = m.release();
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return KETOGPU_ENOMEM;
    } catch (const std::system_error &e) {
        set_last_error(std::string("thread: ") + e.what());
        return KETOGPU_ENOMEM;
    }
    return KETOGPU_OK;
}

void ketogpu_multi_free(ketogpu_multi *m) { delete m; }

size_t ketogpu_multi_size(const ketogpu_multi *m) { return m ? m->eng.size() : 0; }

ketogpu_engine *ketogpu_multi_engine(ketogpu_multi *m, size_t i) {
    return m && i < m->eng.size() ? m->eng[i] : nullptr;
}

int ketogpu_multi_check_ids(ketogpu_multi *m, const uint32_t *roots, const uint32_t *targets, size_t n,
                            uint64_t *allowed_bits, uint64_t *flagged_bits) {
    if (!m || (n && (!roots || !targets || !allowed_bits))) {
        set_last_error("null argument");
        return KETOGPU_EINVAL;
    }
    std::lock_guard<std::mutex> call(m->call_mu);
    {
        std::lock_guard<std::mutex> lk(m->mu);
        m->roots = roots;
        m->targets = targets;
        m->n = n;
        m->allowed = allowed_bits;
        m->flagged = flagged_bits;
        m->pending = m->eng.size();
        m->gen++;
    }
    m->start_cv.notify_all();
    std::unique_lock<std::mutex> lk(m->mu);
    m->done_cv.wait(lk, [&] { return m->pending == 0; });
    for (size_t i = 0; i < m->eng.size(); i++)
        if (m->rc[i]) {
            size_t b = 0, e = 0;
            ketogpu_multi_range(n, m->eng.size(), i, &b, &e);
            // request indices in the engine's message are relative to its range
            set_last_error("device range [" + std::to_string(b) + ", " + std::to_string(e) + "): " + m->err[i]);
            return m->rc[i];
        }
    return KETOGPU_OK;
}

}  // extern "C"
