// host_floor.cpp — where the µs of a small host-buffer call go (VERDICT r03
// next #4).  Standalone lab, linked against the product library; nothing in
// the product uses it.  For each size, median µs per call over `reps` calls:
//   drop_pageable / drop_pinned : s3dlio_fill_controlled_data (the product)
//   fill_only                   : s3dg_fill_controlled on a device buffer + stream sync
//   d2h_only_pinned             : hipMemcpyAsync D2H of the size + stream sync
//   fill_d2h_1s_pinned          : fill + D2H on one stream, hipStreamSynchronize
//   fill_d2h_ev_pinned          : the same, completion by hipEventSynchronize
//   fill_d2h_spin_pinned        : the same, completion by spinning on hipEventQuery
//   fill_to_host_pinned         : the fill kernel stores straight into pinned host memory
//   fill_d2h_1s_pageable        : fill + D2H (HIP stages pageable memory) + sync
//   bounce_memcpy_pageable      : fill + D2H into a pinned bounce + memcpy to the pageable buffer
//   bounce_pipe_pageable        : the same in 4 pieces: memcpy of piece k overlaps D2H of k+1
//   k2h_memcpy_pageable         : fill straight into the pinned bounce + memcpy
//   memcpy_only                 : memcpy of the size, pinned bounce -> pageable
// build: hipcc --offload-arch=gfx950 -O2 -I include tools/r04/host_floor.cpp -L s3dlio_amd -ls3dlio_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "s3dlio_gpu.h"

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)
#define CS(x)                                                                         \
    do {                                                                              \
        int r_ = (x);                                                                 \
        if (r_) {                                                                     \
            fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r_, s3dg_last_error()); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median_us(int reps, const std::function<void()> &f) {
    for (int k = 0; k < 20; ++k) f();
    std::vector<double> t(reps);
    for (int k = 0; k < reps; ++k) {
        const double a = now_us();
        f();
        t[k] = now_us() - a;
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 300;
    s3dg_ctx *ctx = nullptr;
    CS(s3dg_ctx_create(0, &ctx));
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t maxn = 16u << 20;
    void *dev = nullptr, *pin = nullptr;
    CK(hipMalloc(&dev, maxn));
    CK(hipHostMalloc(&pin, maxn, hipHostMallocDefault));
    uint8_t *pg = (uint8_t *)aligned_alloc(4096, maxn);
    memset(pg, 1, maxn);
    memset(pin, 1, maxn);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<size_t> sizes = {64u << 10, 256u << 10, 1u << 20, 4u << 20, 16u << 20};
    const bool rev = argc > 2 && strcmp(argv[2], "rev") == 0;   // largest first (a fresh process's first calls)
    if (rev) std::reverse(sizes.begin(), sizes.end());
    printf("{\"lab\": \"host_floor\", \"reps\": %d, \"order\": \"%s\"}\n", reps, rev ? "rev" : "fwd");
    // helper threads for the multi-threaded copy-out variant: spin on a generation counter
    struct Helper {
        std::atomic<uint64_t> gen{0}, done{0};
        hipEvent_t ev = nullptr;
        uint8_t *dst = nullptr;
        const uint8_t *src = nullptr;
        size_t len = 0;
        std::thread th;
    };
    static Helper hp[3];
    static std::atomic<bool> quit{false};
    for (auto &h : hp)
        h.th = std::thread([&h] {
            uint64_t seen = 0;
            while (!quit.load()) {
                const uint64_t g = h.gen.load(std::memory_order_acquire);
                if (g == seen) continue;
                seen = g;
                (void)hipEventSynchronize(h.ev);
                memcpy(h.dst, h.src, h.len);
                h.done.store(g, std::memory_order_release);
            }
        });
    for (size_t n : sizes) {
        auto fill = [&](void *dst) { CS(s3dg_fill_controlled(ctx, dst, n, 1, 0, 1, 7, s)); };
        std::vector<std::pair<const char *, double>> r;
        r.push_back({"drop_pageable", median_us(reps, [&] { CS(s3dlio_fill_controlled_data(pg, n, 1, 1)); })});
        r.push_back({"drop_pinned", median_us(reps, [&] { CS(s3dlio_fill_controlled_data((uint8_t *)pin, n, 1, 1)); })});
        r.push_back({"fill_only", median_us(reps, [&] { fill(dev); CK(hipStreamSynchronize(s)); })});
        r.push_back({"d2h_only_pinned", median_us(reps, [&] {
                         CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipStreamSynchronize(s));
                     })});
        r.push_back({"fill_d2h_1s_pinned", median_us(reps, [&] {
                         fill(dev);
                         CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipStreamSynchronize(s));
                     })});
        r.push_back({"fill_d2h_ev_pinned", median_us(reps, [&] {
                         fill(dev);
                         CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipEventRecord(ev, s));
                         CK(hipEventSynchronize(ev));
                     })});
        r.push_back({"fill_d2h_spin_pinned", median_us(reps, [&] {
                         fill(dev);
                         CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipEventRecord(ev, s));
                         while (hipEventQuery(ev) == hipErrorNotReady) {
                         }
                     })});
        r.push_back({"fill_to_host_pinned", median_us(reps, [&] { fill(pin); CK(hipStreamSynchronize(s)); })});
        r.push_back({"fill_d2h_1s_pageable", median_us(reps, [&] {
                         fill(dev);
                         CK(hipMemcpyAsync(pg, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipStreamSynchronize(s));
                     })});
        r.push_back({"bounce_memcpy_pageable", median_us(reps, [&] {
                         fill(dev);
                         CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
                         CK(hipStreamSynchronize(s));
                         memcpy(pg, pin, n);
                     })});
        r.push_back({"bounce_pipe_pageable", median_us(reps, [&] {
                         const size_t q = n / 4;
                         hipEvent_t e[4];
                         static hipEvent_t pool[4] = {};
                         if (!pool[0])
                             for (auto &x : pool) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
                         for (int k = 0; k < 4; ++k) e[k] = pool[k];
                         fill(dev);
                         for (int k = 0; k < 4; ++k) {
                             CK(hipMemcpyAsync((uint8_t *)pin + k * q, (uint8_t *)dev + k * q, q, hipMemcpyDeviceToHost, s));
                             CK(hipEventRecord(e[k], s));
                         }
                         for (int k = 0; k < 4; ++k) {
                             while (hipEventQuery(e[k]) == hipErrorNotReady) {
                             }
                             memcpy(pg + k * q, (uint8_t *)pin + k * q, q);
                         }
                     })});
        r.push_back({"k2h_memcpy_pageable", median_us(reps, [&] {
                         fill(pin);
                         CK(hipStreamSynchronize(s));
                         memcpy(pg, pin, n);
                     })});
        r.push_back({"memcpy_only", median_us(reps, [&] { memcpy(pg, pin, n); })});
        // the candidate design: the fill writes the pinned bounce in pieces,
        // the caller copies piece k while pieces k+1.. are generated
        static hipEvent_t pe[8] = {};
        if (!pe[0])
            for (auto &x : pe) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        for (int np : {2, 4, 8}) {
            static char name[3][32];
            char *nm = name[np == 2 ? 0 : (np == 4 ? 1 : 2)];
            snprintf(nm, 32, "k2h_pipe%d_pageable", np);
            const uint64_t nb = n / 4096, per = (nb + np - 1) / np;
            r.push_back({nm, median_us(reps, [&] {
                             for (int k = 0; k < np; ++k) {
                                 const uint64_t b0 = k * per, b1 = std::min<uint64_t>(nb, b0 + per);
                                 CS(s3dg_fill_controlled_range(ctx, (uint8_t *)pin + b0 * 4096, n, b0, b1, 1, 0, 1, 7, s));
                                 CK(hipEventRecord(pe[k], s));
                             }
                             for (int k = 0; k < np; ++k) {
                                 const uint64_t b0 = k * per, b1 = std::min<uint64_t>(nb, b0 + per);
                                 CK(hipEventSynchronize(pe[k]));
                                 memcpy(pg + b0 * 4096, (uint8_t *)pin + b0 * 4096, (b1 - b0) * 4096);
                             }
                         })});
        }
        r.push_back({"k2h_pipe4_mt_pageable", median_us(reps, [&] {
                         const uint64_t nb = n / 4096, per = (nb + 3) / 4;
                         for (int k = 0; k < 4; ++k) {
                             const uint64_t b0 = k * per, b1 = std::min<uint64_t>(nb, b0 + per);
                             CS(s3dg_fill_controlled_range(ctx, (uint8_t *)pin + b0 * 4096, n, b0, b1, 1, 0, 1, 7, s));
                             CK(hipEventRecord(pe[k], s));
                             if (k) {
                                 Helper &h = hp[k - 1];
                                 h.ev = pe[k];
                                 h.dst = pg + b0 * 4096;
                                 h.src = (uint8_t *)pin + b0 * 4096;
                                 h.len = (b1 - b0) * 4096;
                                 h.gen.fetch_add(1, std::memory_order_release);
                             }
                         }
                         CK(hipEventSynchronize(pe[0]));
                         memcpy(pg, pin, std::min<uint64_t>(nb, per) * 4096);
                         for (auto &h : hp)
                             while (h.done.load(std::memory_order_acquire) != h.gen.load()) {
                             }
                     })});
        if (n >= (1u << 20)) {
            r.push_back({"dgen_dev", median_us(reps, [&] {
                             CS(s3dg_dgen_fill(ctx, dev, n, 0, n >> 20, 1, 0, 1, 9, s));
                             CK(hipStreamSynchronize(s));
                         })});
            r.push_back({"dgen_to_host_pinned", median_us(reps, [&] {
                             CS(s3dg_dgen_fill(ctx, pin, n, 0, n >> 20, 1, 0, 1, 9, s));
                             CK(hipStreamSynchronize(s));
                         })});
        }
        printf("{\"bytes\": %zu", n);
        for (auto &kv : r) printf(", \"%s\": %.1f", kv.first, kv.second);
        printf("}\n");
        fflush(stdout);
    }
    quit.store(true);
    for (auto &h : hp) h.th.join();
    return 0;
}
