// gather_probe.hip — what does one random head read cost on MI355X?  A microbenchmark for
// plan label's first stage (device_engine.hip label_unit): every request reads TWO heads of
// W bytes at random W-aligned places of a table far larger than L2 + Infinity Cache, four
// lanes per request (one DPP quad), 16 requests per wave, and stores one bit per request.
// Variants:
//   W = 32, 64, 128, 256 bytes per head (whole-head reads)
//   split: 128-byte heads, the first 64 bytes read always and the second 64 bytes read
//          (a dependent second read) only for the share `p` of requests (by hash)
// Prints one JSON line per variant: ms per 1M requests, requests/s, head bytes/s.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/gather_probe tools/gather_probe.hip
//   ./tools/gather_probe [table_GB=4] [requests=1000000]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 30, x *= 0xbf58476d1ce4e5b9ull, x ^= x >> 27, x *= 0x94d049bb133111ebull, x ^= x >> 31;
    return x;
}

// W bytes per head; lane `sub` reads W/4 bytes
template <int W>
__device__ __forceinline__ uint32_t read_head(const uint32_t *T, uint64_t slot, uint32_t sub) {
    const uint32_t *h = T + slot * (W / 4);
    if constexpr (W == 32) {
        const uint2 a = reinterpret_cast<const uint2 *>(h)[sub];
        return a.x ^ a.y;
    } else {
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < W / 64; k++) {
            const uint4 a = reinterpret_cast<const uint4 *>(h)[(W / 64) * sub + k];
            s ^= a.x ^ a.y ^ a.z ^ a.w;
        }
        return s;
    }
}

template <int W>
__global__ __launch_bounds__(64) void probe_kernel(const uint32_t *T, uint64_t slots, const uint32_t *rq, uint64_t n,
                                                   uint32_t *out) {
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint64_t i = (uint64_t)blockIdx.x * 16 + q;
    uint32_t a = 0, b = 0;
    if (lane < 16 && (uint64_t)blockIdx.x * 16 + lane < n) a = rq[2 * ((uint64_t)blockIdx.x * 16 + lane)],
                                                                b = rq[2 * ((uint64_t)blockIdx.x * 16 + lane) + 1];
    a = __shfl(a, q, 64), b = __shfl(b, q, 64);
    uint32_t v = 0;
    if (i < n) v = read_head<W>(T, a % slots, sub) ^ read_head<W>(T, b % slots, sub);
    const uint64_t bits = __ballot((v & 0xF) == 3);
    if (lane == 0) reinterpret_cast<uint16_t *>(out)[blockIdx.x] = (uint16_t)(bits ^ (bits >> 16));
}

// 128-byte heads: the first 64 bytes always, the second 64 only for requests whose hash < p
__global__ __launch_bounds__(64) void split_kernel(const uint32_t *T, uint64_t slots, const uint32_t *rq, uint64_t n,
                                                   uint32_t *out, uint32_t permille) {
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint64_t i = (uint64_t)blockIdx.x * 16 + q;
    uint32_t a = 0, b = 0;
    if (lane < 16 && (uint64_t)blockIdx.x * 16 + lane < n) a = rq[2 * ((uint64_t)blockIdx.x * 16 + lane)],
                                                                b = rq[2 * ((uint64_t)blockIdx.x * 16 + lane) + 1];
    a = __shfl(a, q, 64), b = __shfl(b, q, 64);
    uint32_t v = 0;
    const uint64_t sa = a % slots, sb = b % slots;
    if (i < n) {
        const uint4 x = reinterpret_cast<const uint4 *>(T + sa * 32)[sub];
        const uint4 y = reinterpret_cast<const uint4 *>(T + sb * 32)[sub];
        v = x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w;
        // the decision to read on depends on the first read (as a count word would)
        const uint32_t c = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x.x), 0, 0xf, 0xf, false);
        if ((mix(i ^ c) % 1000) < permille) {
            const uint4 z = reinterpret_cast<const uint4 *>(T + sa * 32 + 16)[sub];
            v ^= z.x ^ z.y ^ z.z ^ z.w;
        }
    }
    const uint64_t bits = __ballot((v & 0xF) == 3);
    if (lane == 0) reinterpret_cast<uint16_t *>(out)[blockIdx.x] = (uint16_t)(bits ^ (bits >> 16));
}

// side A: WA-byte heads of a small table (cache-resident?), side B: 128-byte heads of the big
// table, B read non-temporally when NT
template <int WA, bool NT>
__global__ __launch_bounds__(64) void two_kernel(const uint32_t *A, uint64_t slots_a, const uint32_t *T, uint64_t slots,
                                                 const uint32_t *rq, uint64_t n, uint32_t *out) {
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint64_t i = (uint64_t)blockIdx.x * 16 + q;
    uint32_t a = 0, b = 0;
    if (lane < 16 && (uint64_t)blockIdx.x * 16 + lane < n) a = rq[2 * ((uint64_t)blockIdx.x * 16 + lane)],
                                                                b = rq[2 * ((uint64_t)blockIdx.x * 16 + lane) + 1];
    a = __shfl(a, q, 64), b = __shfl(b, q, 64);
    uint32_t v = 0;
    if (i < n) {
        v = read_head<WA>(A, a % slots_a, sub);
        const uint4 *p = reinterpret_cast<const uint4 *>(T + (b % slots) * 32) + sub * 2;
        if (NT) {
            typedef unsigned int u4v __attribute__((ext_vector_type(4)));
            const u4v *pv = reinterpret_cast<const u4v *>(p);
            const u4v x = __builtin_nontemporal_load(pv), y = __builtin_nontemporal_load(pv + 1);
            v ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w;
        } else {
            const uint4 x = p[0], y = p[1];
            v ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w;
        }
    }
    const uint64_t bits = __ballot((v & 0xF) == 3);
    if (lane == 0) reinterpret_cast<uint16_t *>(out)[blockIdx.x] = (uint16_t)(bits ^ (bits >> 16));
}

// 128-byte heads, two per request; WPG waves per workgroup, each wave U units (of 16
// requests) with all of its units' loads issued before any is used; grid-stride persistent
// when the grid is smaller than the units
template <int WPG, int U>
__global__ __launch_bounds__(64 * WPG) void multi_kernel(const uint32_t *T, uint64_t slots, const uint32_t *rq, uint64_t n,
                                                         uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, q = lane >> 2, sub = lane & 3, wave = threadIdx.x >> 6;
    const uint64_t units = (n + 15) / 16;
    for (uint64_t u0 = ((uint64_t)blockIdx.x * WPG + wave) * U; u0 < units; u0 += (uint64_t)gridDim.x * WPG * U) {
        uint32_t a[U], b[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const uint64_t j = (u0 + k) * 16 + lane;
            a[k] = b[k] = 0;
            if (lane < 16 && j < n) a[k] = rq[2 * j], b[k] = rq[2 * j + 1];
            a[k] = __shfl(a[k], q, 64), b[k] = __shfl(b[k], q, 64);
        }
        uint4 x[U], y[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            x[k] = reinterpret_cast<const uint4 *>(T + (a[k] % slots) * 32)[sub * 2];
            y[k] = reinterpret_cast<const uint4 *>(T + (b[k] % slots) * 32)[sub * 2 + 1];
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const uint32_t v = x[k].x ^ x[k].y ^ x[k].z ^ x[k].w ^ y[k].x ^ y[k].y ^ y[k].z ^ y[k].w;
            const uint64_t bits = __ballot((v & 0xF) == 3);
            if (lane == 0 && u0 + k < units) reinterpret_cast<uint16_t *>(out)[u0 + k] = (uint16_t)(bits ^ (bits >> 16));
        }
    }
}

template <class F>
static float time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int k = 0; k < 3; k++) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int k = 0; k < reps; k++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 4.0;
    const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1000000;
    const uint64_t bytes = (uint64_t)(gb * (1ull << 30)) / 256 * 256;
    uint32_t *T, *rq, *out;
    CK(hipMalloc(&T, bytes));
    CK(hipMemset(T, 0x5a, bytes));
    std::vector<uint32_t> h(2 * n);
    uint64_t s = 88172645463325252ull;
    for (auto &x : h) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        x = (uint32_t)(s >> 17);
    }
    CK(hipMalloc(&rq, 8 * n));
    CK(hipMemcpy(rq, h.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, n / 8 + 64));
    const uint32_t grid = (uint32_t)((n + 15) / 16);
    const int reps = 20;
    auto report = [&](const char *name, int w, double ms, double head_bytes) {
        printf("{\"variant\": \"%s\", \"head_bytes\": %d, \"table_GB\": %.1f, \"requests\": %llu, \"ms\": %.5f, "
               "\"ms_per_1M\": %.5f, \"requests_per_s\": %.4g, \"head_GBps\": %.1f}\n",
               name, w, gb, (unsigned long long)n, ms, ms * 1e6 / (double)n, (double)n / (ms * 1e-3),
               head_bytes * (double)n / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
#define RUN(W)                                                                                        \
    {                                                                                                 \
        const uint64_t slots = bytes / W;                                                             \
        float ms = time_ms([&] { probe_kernel<W><<<grid, 64>>>(T, slots, rq, n, out); }, reps);       \
        CK(hipGetLastError());                                                                        \
        report("whole", W, ms, 2.0 * W);                                                              \
    }
    RUN(32) RUN(64) RUN(128) RUN(256)
    for (uint32_t p : {0u, 100u, 250u, 500u, 1000u}) {
        const uint64_t slots = bytes / 128;
        float ms = time_ms([&] { split_kernel<<<grid, 64>>>(T, slots, rq, n, out, p); }, reps);
        CK(hipGetLastError());
        char name[64];
        snprintf(name, sizeof name, "split_p%u", p);
        report(name, 128, ms, 2.0 * 64 + 64.0 * p / 1000.0);
    }
    {
        const uint64_t slots = bytes / 128, units = (n + 15) / 16;
#define MULTI(WPG, U, GRID)                                                                                     \
    {                                                                                                         \
        const uint32_t g = GRID ? GRID : (uint32_t)((units + WPG * U - 1) / (WPG * U));                        \
        float ms = time_ms([&] { multi_kernel<WPG, U><<<g, 64 * WPG>>>(T, slots, rq, n, out); }, reps);        \
        CK(hipGetLastError());                                                                                \
        char name[64];                                                                                        \
        snprintf(name, sizeof name, "multi_wpg%d_u%d_grid%u", WPG, U, g);                                     \
        report(name, 128, ms, 256.0);                                                                         \
    }
        MULTI(1, 1, 0) MULTI(4, 1, 0) MULTI(1, 2, 0) MULTI(1, 4, 0) MULTI(4, 2, 0) MULTI(4, 4, 0)
        MULTI(1, 1, 8192) MULTI(1, 1, 4096) MULTI(4, 1, 2048) MULTI(1, 2, 4096) MULTI(1, 4, 2048) MULTI(4, 2, 1024)
    }
    for (uint64_t mb : {8ull, 32ull, 128ull, 512ull, 2048ull}) {  // both heads from a table of mb MB
        const uint64_t slots = (mb << 20) / 128;
        float ms = time_ms([&] { probe_kernel<128><<<grid, 64>>>(T, slots, rq, n, out); }, reps);
        CK(hipGetLastError());
        char name[64];
        snprintf(name, sizeof name, "table_%lluMB", (unsigned long long)mb);
        report(name, 128, ms, 256.0);
    }
    for (uint64_t mb : {32ull, 67ull, 134ull, 269ull, 538ull}) {
        const uint64_t ab = mb << 20;
#define TWO(WA, NT)                                                                                              \
    {                                                                                                            \
        float ms = time_ms([&] { two_kernel<WA, NT><<<grid, 64>>>(T + bytes / 8, ab / WA, T, bytes / 2 / 128, rq, n, out); }, \
                           reps);                                                                                \
        CK(hipGetLastError());                                                                                   \
        char name[64];                                                                                           \
        snprintf(name, sizeof name, "two_A%lluMB_nt%d", (unsigned long long)mb, (int)NT);                       \
        report(name, WA, ms, WA + 128.0);                                                                        \
    }
        TWO(64, false) TWO(128, false) TWO(64, true) TWO(128, true)
    }
    CK(hipFree(T));
    CK(hipFree(rq));
    CK(hipFree(out));
    return 0;
}
