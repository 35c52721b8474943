// s3dg_generator.cpp — streaming object generator over the device keystream
// kernel: the drop-in behind s3dlio's dgen-data-backed surface
//   Rust:  DataGenerator / ObjectGen (src/data_gen.rs:253-371),
//          ObjectGenAlt (src/data_gen_alt.rs:89-149), generate_controlled_data_alt (:66-80)
//   PyO3:  Generator (src/python_api/python_datagen_api.rs:270-365),
//          generate_data / generate_into_buffer (:49-200)
// dgen-data 0.2.4 (the reference's engine) is not in the checkout, so the byte
// stream is build-defined ("DG1") and meets the reference
// tests' statistical contract; parity unpinned.
//
// DG1, for an object of `size` bytes, 1 MiB blocks (DGEN_BLOCK_SIZE,
// src/constants.rs:348), U = unique_blocks(nblocks, dedup):
//   block i = Xoshiro256PlusPlus::seed_from_u64(seed ^ ((i % U) * phi)).fill_bytes(L_i)
//             with its first floor(L_i * f_num / f_den) bytes zeroed (compress).
// Generation is positional, so output is independent of fill_chunk sizes.
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <time.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

extern "C" int s3dg_internal_fail(int code, const char *msg);   // s3dg_capi.cpp
extern "C" s3dg_ctx *s3dg_internal_default_ctx(int *err);       // s3dg_capi.cpp
extern "C" int s3dg_internal_ctx_device(s3dg_ctx *c, int *dev);  // s3dg_capi.cpp

// Device staging for host-buffer generation: two 64 MiB chunks + two
// streams.  Pooled process-wide so short-lived generators (generate_data on
// small sizes) do not pay hipMalloc / stream creation per call.
struct Scratch {
    void *buf[2] = {nullptr, nullptr};
    hipStream_t st[2] = {nullptr, nullptr};
};

struct s3dg_gen {
    s3dg_ctx *ctx = nullptr;
    uint64_t size = 0, dedup = 1, seed = 0, pos = 0;
    uint32_t f_num = 0, f_den = 1;
    Scratch *sc = nullptr;
    std::mutex mu;
};

namespace {

using namespace s3dg;

constexpr uint64_t kMaxScratchBlocks = 64;   // 64 MiB per device chunk

uint64_t unseeded_entropy() {
    // like DataGenerator::new(None): time + per-thread counter (src/data_gen.rs:271-291)
    static std::atomic<uint64_t> counter{0};
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const uint64_t base = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    return base + counter.fetch_add(1) * 0x9E3779B97F4A7C15ull;
}

#define GEN_HIP(expr, what)                                                          \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess)                                                        \
            return s3dg_internal_fail(S3DG_EHIP, (std::string(what) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

std::mutex pool_mu;
std::vector<Scratch *> pool;    // idle scratch sets

int acquire_scratch(s3dg_gen *g) {
    if (g->sc) return S3DG_OK;
    {
        std::lock_guard<std::mutex> lk(pool_mu);
        if (!pool.empty()) {
            g->sc = pool.back();
            pool.pop_back();
            return S3DG_OK;
        }
    }
    Scratch *sc = new Scratch();
    for (int k = 0; k < 2; ++k) {
        if (hipMalloc(&sc->buf[k], kMaxScratchBlocks * kDgenBlock) != hipSuccess ||
            hipStreamCreateWithFlags(&sc->st[k], hipStreamNonBlocking) != hipSuccess) {
            for (int q = 0; q < 2; ++q) {
                if (sc->buf[q]) (void)hipFree(sc->buf[q]);
                if (sc->st[q]) (void)hipStreamDestroy(sc->st[q]);
            }
            delete sc;
            return s3dg_internal_fail(S3DG_EHIP, "generator scratch allocation failed");
        }
    }
    g->sc = sc;
    return S3DG_OK;
}

void release_scratch(s3dg_gen *g) {
    if (!g->sc) return;
    for (int k = 0; k < 2; ++k) (void)hipStreamSynchronize(g->sc->st[k]);
    std::lock_guard<std::mutex> lk(pool_mu);
    pool.push_back(g->sc);
    g->sc = nullptr;
}

// Bytes [pos, pos+n) of the object into host `buf`: covering 1 MiB blocks are
// generated into two device chunks on two streams (chunk k+1's kernel
// overlaps chunk k's D2H), then exactly the requested bytes are copied out.
int fill_range(s3dg_gen *g, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (n == 0) return S3DG_OK;
    // the caller's thread may have another device current: scratch is
    // allocated (and kernels launched) on the context's device
    int dev = 0;
    if (int r = s3dg_internal_ctx_device(g->ctx, &dev)) return r;
    DeviceScope ds(dev);
    if (!ds.ok()) return s3dg_internal_fail(S3DG_EHIP, "hipSetDevice");
    if (int r = acquire_scratch(g)) return r;
    Scratch *sc = g->sc;
    const uint64_t b0 = pos / kDgenBlock, b1 = (pos + n + kDgenBlock - 1) / kDgenBlock;
    int k = 0;
    for (uint64_t pb = b0; pb < b1; pb += kMaxScratchBlocks, ++k) {
        const uint64_t pe = pb + kMaxScratchBlocks < b1 ? pb + kMaxScratchBlocks : b1;
        const int sl = k & 1;
        if (int r = s3dg_dgen_fill(g->ctx, sc->buf[sl], g->size, pb, pe, g->dedup, g->f_num,
                                   g->f_den, g->seed, sc->st[sl]))
            return r;
        const uint64_t lo = pb * kDgenBlock > pos ? pb * kDgenBlock : pos;
        const uint64_t hi = pe * kDgenBlock < pos + n ? pe * kDgenBlock : pos + n;
        GEN_HIP(hipMemcpyAsync(buf + (lo - pos), (uint8_t *)sc->buf[sl] + (lo - pb * kDgenBlock),
                               hi - lo, hipMemcpyDeviceToHost, sc->st[sl]),
                "hipMemcpyAsync(D2H)");
    }
    GEN_HIP(hipStreamSynchronize(sc->st[0]), "hipStreamSynchronize");
    GEN_HIP(hipStreamSynchronize(sc->st[1]), "hipStreamSynchronize");
    return S3DG_OK;
}

}  // namespace

extern "C" {

int s3dg_gen_create_ratio(uint64_t size, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                          int has_seed, uint64_t seed, s3dg_gen **out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *out = nullptr;
    if (f_den == 0 || f_num >= f_den) return s3dg_internal_fail(S3DG_EINVAL, "need f_num < f_den");
    int err = 0;
    s3dg_ctx *ctx = s3dg_internal_default_ctx(&err);
    if (!ctx) return err;
    s3dg_gen *g = new s3dg_gen();
    g->ctx = ctx;
    g->size = size;
    g->dedup = dedup == 0 ? 1 : dedup;       // .max(1), src/data_gen_alt.rs:108
    g->f_num = f_num;
    g->f_den = f_den;
    g->seed = has_seed ? seed : unseeded_entropy();
    *out = g;
    return S3DG_OK;
}

int s3dg_gen_create(uint64_t size, uint64_t dedup, uint64_t compress, int has_seed, uint64_t seed,
                    s3dg_gen **out) {
    uint32_t fn, fd;
    if (int r = s3dg_compress_ratio(compress, &fn, &fd)) return r;   // .max(1): c<=1 -> (0,1)
    return s3dg_gen_create_ratio(size, dedup, fn, fd, has_seed, seed, out);
}

int s3dg_gen_destroy(s3dg_gen *g) {
    if (!g) return S3DG_OK;
    release_scratch(g);
    delete g;
    return S3DG_OK;
}

int s3dg_gen_fill_chunk(s3dg_gen *g, uint8_t *buf, uint64_t cap, uint64_t *written) {
    if (!g || !written) return s3dg_internal_fail(S3DG_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    *written = 0;
    const uint64_t n = cap < g->size - g->pos ? cap : g->size - g->pos;
    if (n == 0) return S3DG_OK;                                     // complete: 0 bytes
    if (!buf) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    if (int r = fill_range(g, buf, g->pos, n)) return r;
    g->pos += n;
    *written = n;
    return S3DG_OK;
}

int s3dg_gen_fill_at(s3dg_gen *g, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (!g) return s3dg_internal_fail(S3DG_EINVAL, "null generator");
    if (pos > g->size || n > g->size - pos) return s3dg_internal_fail(S3DG_EINVAL, "range past the object");
    std::lock_guard<std::mutex> lk(g->mu);
    return fill_range(g, buf, pos, n);
}

int s3dg_gen_is_complete(s3dg_gen *g) { return g && g->pos >= g->size; }
uint64_t s3dg_gen_position(s3dg_gen *g) { return g ? g->pos : 0; }
uint64_t s3dg_gen_total_size(s3dg_gen *g) { return g ? g->size : 0; }
uint64_t s3dg_gen_seed(s3dg_gen *g) { return g ? g->seed : 0; }
int s3dg_gen_reset(s3dg_gen *g) {
    if (!g) return s3dg_internal_fail(S3DG_EINVAL, "null generator");
    std::lock_guard<std::mutex> lk(g->mu);
    g->pos = 0;
    return S3DG_OK;
}

int s3dg_generate_data(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t compress, int has_seed,
                       uint64_t seed) {
    if (size == 0) return S3DG_OK;
    s3dg_gen *g = nullptr;
    if (int r = s3dg_gen_create(size, dedup, compress, has_seed, seed, &g)) return r;
    uint64_t w = 0;
    int r = s3dg_gen_fill_chunk(g, buf, size, &w);
    s3dg_gen_destroy(g);
    return r;
}

}  // extern "C"
