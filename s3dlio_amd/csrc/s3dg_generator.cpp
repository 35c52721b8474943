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

// Host staging (two 64 MiB device chunks + two streams) comes from the host
// slot pool (s3dg_host.cpp): the generator takes a slot round-robin at
// creation and holds one staging set of that slot from its first fill to its
// destruction, so short-lived generators reuse pooled sets instead of paying
// hipMalloc / stream creation per call, and concurrent generators run on
// different GPUs.
struct s3dg_gen {
    int slot = 0;
    uint64_t size = 0, dedup = 1, seed = 0, pos = 0;
    uint32_t f_num = 0, f_den = 1;
    s3dg::HostStaging *sg = nullptr;
    std::mutex mu;
};

namespace {

using namespace s3dg;

uint64_t unseeded_entropy() {
    // like DataGenerator::new(None): time + per-thread counter (src/data_gen.rs:271-291)
    static std::atomic<uint64_t> counter{0};
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const uint64_t base = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    return base + counter.fetch_add(1) * 0x9E3779B97F4A7C15ull;
}

// Bytes [pos, pos+n) of the object into host `buf` (s3dg_host.cpp host_run:
// covering 1 MiB blocks through the staging chunks; large requests split
// over the slots).
int fill_range(s3dg_gen *g, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (n == 0) return S3DG_OK;
    if (!g->sg)
        if (int r = host_staging_acquire(g->slot, &g->sg)) return r;
    HostJob J;
    J.dgen = true;
    J.obj_len = g->size;
    J.entropy = g->seed;
    J.dedup = g->dedup;
    J.f_num = g->f_num;
    J.f_den = g->f_den;
    return host_run_split(g->sg, J, buf, pos, n);
}

}  // namespace

extern "C" {

int s3dg_gen_create_ratio(uint64_t size, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                          int has_seed, uint64_t seed, s3dg_gen **out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *out = nullptr;
    if (f_den == 0 || f_num >= f_den) return s3dg_internal_fail(S3DG_EINVAL, "need f_num < f_den");
    int slot = 0;
    if (int r = host_next_slot(&slot)) return r;
    s3dg_gen *g = new s3dg_gen();
    g->slot = slot;
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
    host_staging_release(g->sg);
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
int s3dg_gen_slot(s3dg_gen *g) { return g ? g->slot : -1; }
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
