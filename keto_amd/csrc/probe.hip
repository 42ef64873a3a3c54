// probe.hip — the random-line ceiling of plan label's first stage, measured live
// (ketogpu_probe_random_lines, include/ketogpu.h "diagnostics").  A check reads one head of
// its target and one of its root: two random 128-byte lines of tables far larger than L2 and
// the Infinity Cache, plus 8 bytes of request.  This kernel does exactly that and nothing
// else — 16 requests per wave, four lanes per request, both lines in flight at once, one
// result bit per request — so its time per launch is what label_kernel's reads alone cost
// on the same device (tools/gather_probe.hip explores the shapes: profiles/r06/probe/).
// bench.py reports label_kernel's time against it (roofline.line_ceiling).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ketogpu.h"

namespace {

__global__ __launch_bounds__(64) void probe_lines_kernel(const uint32_t *table, uint64_t lines, const uint32_t *rq,
                                                         uint64_t n, uint16_t *out) {
    const uint32_t lane = threadIdx.x, q = lane >> 2, sub = lane & 3;
    const uint64_t i0 = (uint64_t)blockIdx.x * 16;
    uint32_t a = 0, b = 0;
    if (lane < 16 && i0 + lane < n) a = rq[2 * (i0 + lane)], b = rq[2 * (i0 + lane) + 1];
    a = (uint32_t)__shfl((int)a, (int)q, 64);
    b = (uint32_t)__shfl((int)b, (int)q, 64);
    uint32_t v = 0;
    if (i0 + q < n) {
        const uint4 *x = reinterpret_cast<const uint4 *>(table + (a % lines) * 32) + 2 * sub;
        const uint4 *y = reinterpret_cast<const uint4 *>(table + (b % lines) * 32) + 2 * sub;
        const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
        v = x0.x ^ x0.y ^ x0.z ^ x0.w ^ x1.x ^ x1.y ^ x1.z ^ x1.w ^ y0.x ^ y0.y ^ y0.z ^ y0.w ^ y1.x ^ y1.y ^ y1.z ^ y1.w;
    }
    const uint64_t bits = __ballot((v & 0xF) == 3);
    if (lane == 0) out[blockIdx.x] = (uint16_t)(bits ^ (bits >> 16) ^ (bits >> 32) ^ (bits >> 48));
}

}  // namespace

extern "C" int ketogpu_probe_random_lines(int device, uint64_t table_bytes, uint64_t requests, int reps,
                                          double *ms_per_launch) {
    if (!ms_per_launch || requests == 0 || reps <= 0 || table_bytes < (1u << 20)) return KETOGPU_EINVAL;
    *ms_per_launch = 0;
    if (hipSetDevice(device) != hipSuccess) return KETOGPU_EDEVICE;
    const uint64_t lines = table_bytes / 128;
    uint32_t *table = nullptr, *rq = nullptr;
    uint16_t *out = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = KETOGPU_OK;
    auto ok = [&](hipError_t e) {
        if (e != hipSuccess && rc == KETOGPU_OK) rc = e == hipErrorOutOfMemory ? KETOGPU_ENOMEM : KETOGPU_EDEVICE;
        return rc == KETOGPU_OK;
    };
    const uint64_t grid = (requests + 15) / 16;
    if (ok(hipMalloc(&table, lines * 128)) && ok(hipMalloc(&rq, 8 * requests)) && ok(hipMalloc(&out, 2 * grid)) &&
        ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) && ok(hipEventCreate(&e0)) && ok(hipEventCreate(&e1)) &&
        ok(hipMemsetAsync(table, 0x5a, lines * 128, s))) {
        // random request ids (xorshift on the host: the same sequence every run)
        uint32_t *h = nullptr;
        if (ok(hipHostMalloc(&h, 8 * requests, hipHostMallocDefault))) {
            uint64_t x = 88172645463325252ull;
            for (uint64_t k = 0; k < 2 * requests; k++) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                h[k] = (uint32_t)(x >> 17);
            }
            if (ok(hipMemcpyAsync(rq, h, 8 * requests, hipMemcpyHostToDevice, s)) && ok(hipStreamSynchronize(s))) {
                for (int k = 0; k < 3 && rc == KETOGPU_OK; k++)
                    probe_lines_kernel<<<dim3((unsigned)grid), dim3(64), 0, s>>>(table, lines, rq, requests, out);
                ok(hipGetLastError());
                if (ok(hipEventRecord(e0, s))) {
                    for (int k = 0; k < reps && rc == KETOGPU_OK; k++)
                        probe_lines_kernel<<<dim3((unsigned)grid), dim3(64), 0, s>>>(table, lines, rq, requests, out);
                    ok(hipGetLastError());
                    float ms = 0;
                    if (ok(hipEventRecord(e1, s)) && ok(hipEventSynchronize(e1)) && ok(hipEventElapsedTime(&ms, e0, e1)))
                        *ms_per_launch = ms / reps;
                }
            }
            (void)hipHostFree(h);
        }
    }
    if (s) (void)hipStreamSynchronize(s);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    for (void *p : {(void *)table, (void *)rq, (void *)out})
        if (p) (void)hipFree(p);
    return rc;
}
