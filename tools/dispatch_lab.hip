// tools/dispatch_lab.hip — where the ~3.7 us per call of the device
// single-call path (bench.py configs 11-13: s3dg_fill_controlled on one
// 1/4/16 MiB buffer, back to back on one stream) goes.
// Back-to-back launches on one stream, each timed three ways:
//   * host enqueue time per call (the loop's wall clock before the sync),
//   * wall time per call to the end of the sync,
//   * HIP-event time per call over the whole loop;
// for (a) an empty kernel of 1 workgroup, (b) an empty kernel of 256
// workgroups, (c) a plain store kernel writing the same 1 MiB as 256
// workgroups of 128 threads (16-B stores), and (d) s3dg_fill_controlled itself
// (1, 4, 16 MiB) through the library.  In-bounds by construction: (c)'s grid
// covers exactly the buffer.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_native/dispatch_lab tools/dispatch_lab.hip \
//         -I include -L s3dlio_amd -ls3dlio_amd -Wl,-rpath,'$ORIGIN/../../s3dlio_amd'
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

#include "s3dlio_gpu.h"

__global__ void k_empty() {}

__global__ __launch_bounds__(128) void k_store(uint4 *dst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;   // 256 uint4 = 4 KiB per workgroup
    const uint4 v = {(uint32_t)i, 1u, 2u, 3u};
    dst[i] = v;
    dst[i + 128] = v;
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                      \
        }                                                                  \
    } while (0)

using clk = std::chrono::steady_clock;

template <class F>
static int timed(const char *name, int calls, hipStream_t s, F f) {
    for (int k = 0; k < 200; ++k)
        if (f()) return 1;
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const auto t0 = clk::now();
    CK(hipEventRecord(a, s));
    for (int k = 0; k < calls; ++k)
        if (f()) return 1;
    CK(hipEventRecord(b, s));
    const auto t1 = clk::now();
    CK(hipEventSynchronize(b));
    const auto t2 = clk::now();
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
    const double wall = std::chrono::duration<double, std::micro>(t2 - t0).count() / calls;
    printf("{\"case\": \"%s\", \"calls\": %d, \"host_enqueue_us_per_call\": %.3f, \"wall_us_per_call\": %.3f, "
           "\"event_us_per_call\": %.3f}\n",
           name, calls, enq, wall, ms * 1e3 / calls);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    const int calls = 20000;
    hipStream_t s;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const uint64_t MiB = 1ull << 20;
    uint8_t *buf = nullptr;
    CK(hipMalloc(&buf, 16 * MiB));
    s3dg_ctx *ctx = nullptr;
    if (s3dg_ctx_create(0, &ctx)) {
        fprintf(stderr, "s3dg_ctx_create: %s\n", s3dg_last_error());
        return 1;
    }
    int r = 0;
    r |= timed("empty kernel, 1 workgroup", calls, s, [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        return (int)hipGetLastError();
    });
    r |= timed("empty kernel, 256 workgroups of 128", calls, s, [&] {
        hipLaunchKernelGGL(k_empty, dim3(256), dim3(128), 0, s);
        return (int)hipGetLastError();
    });
    r |= timed("plain 16-B store kernel, 1 MiB (256 x 128)", calls, s, [&] {
        hipLaunchKernelGGL(k_store, dim3(256), dim3(128), 0, s, (uint4 *)buf);
        return (int)hipGetLastError();
    });
    for (uint64_t mib : {1ull, 4ull, 16ull}) {
        char name[96];
        snprintf(name, sizeof name, "s3dg_fill_controlled, %llu MiB", (unsigned long long)mib);
        r |= timed(name, mib == 16 ? calls / 4 : calls, s, [&] {
            return s3dg_fill_controlled(ctx, buf, mib * MiB, 1, 0, 1, 7, s);
        });
    }
    if (r) fprintf(stderr, "error: %s\n", s3dg_last_error());
    CK(hipStreamSynchronize(s));
    s3dg_ctx_destroy(ctx);
    CK(hipFree(buf));
    CK(hipStreamDestroy(s));
    printf("dispatch_lab %s\n", r ? "failed" : "ok");
    return r;
}
