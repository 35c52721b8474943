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
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

// Host staging (two 64 MiB device chunks + two streams) comes from the host
// slot pool (s3dg_host.cpp): the generator takes a slot round-robin at
// creation and holds one staging set of that slot from its first fill to its
// destruction, so short-lived generators reuse pooled sets instead of paying
// hipMalloc / stream creation per call, and concurrent generators run on
// different GPUs.
//
// Read-ahead.  The reference's streaming callers pull
// small chunks: StreamingDataWriter::generate_remaining 64 KiB
// (src/streaming_writer.rs:111-116), generate_controlled_data_streaming
// Config::chunk_size = 256 KiB (src/data_gen.rs:232-249, src/config.rs:131).
// A chunk smaller than a ring half is served by memcpy from a pinned host ring
// of two halves on the slot's NUMA node: half h holds the object's bytes
// [h*half, (h+1)*half), written by the keystream kernel directly (no copy
// engine).  Entering half h starts half h+1 in the other slot of the ring, so
// the GPU generates ahead while the caller copies.  Generation is positional,
// so the bytes are those of the synchronous path for any chunk sizes.
// Larger chunks, fill_at and one-shot generate_data take the synchronous path.
struct s3dg_gen {
    int slot = 0, device = 0;
    uint64_t size = 0, dedup = 1, seed = 0;
    std::atomic<uint64_t> pos{0};   // read without the mutex by is_complete / position
    uint32_t f_num = 0, f_den = 1;
    s3dg::HostStaging *sg = nullptr;
    s3dg::HostRing *ring = nullptr;
    bool ring_none = false;          // the ring pool said no: synchronous path
    int64_t held[2] = {-1, -1};      // half index in each ring slot (-1: none)
    bool pending[2] = {false, false};
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

// Ring half size: S3DLIO_GEN_RING_HALF_MIB (1..64, default 4; 0 = no read-ahead).
uint64_t ring_half() {
    static const uint64_t v = [] {
        const char *e = getenv("S3DLIO_GEN_RING_HALF_MIB");
        long m = e && *e ? strtol(e, nullptr, 10) : 4;
        if (m < 0) m = 0;
        if (m > 64) m = 64;
        return (uint64_t)m * kDgenBlock;
    }();
    return v;
}

HostJob dgen_job(const s3dg_gen *g) {
    HostJob J;
    J.dgen = true;
    J.obj_len = g->size;
    J.entropy = g->seed;
    J.dedup = g->dedup;
    J.f_num = g->f_num;
    J.f_den = g->f_den;
    return J;
}

// Bytes [pos, pos+n) of the object into host `buf` (s3dg_host.cpp host_run:
// covering 1 MiB blocks; large requests split over the slots).
int fill_range(s3dg_gen *g, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (n == 0) return S3DG_OK;
    if (!g->sg)
        if (int r = host_staging_acquire(g->slot, &g->sg)) return r;
    return host_run_split(g->sg, dgen_job(g), buf, pos, n);
}

// Wait for ring slot q's half (if in flight).
int ring_wait(s3dg_gen *g, int q) {
    if (!g->pending[q]) return S3DG_OK;
    g->pending[q] = false;
    const hipError_t e = hipEventSynchronize(g->ring->ev[q]);
    if (e != hipSuccess) {
        g->held[q] = -1;
        return s3dg_internal_fail(S3DG_EHIP, (std::string("read-ahead: ") + hipGetErrorString(e)).c_str());
    }
    return S3DG_OK;
}

// Make ring slot h&1 hold half h (launch it unless it is there or on its way).
int ring_start(s3dg_gen *g, uint64_t h) {
    const uint64_t H = g->ring->half;
    if (h * H >= g->size) return S3DG_OK;
    const int q = (int)(h & 1);
    if (g->held[q] == (int64_t)h) return S3DG_OK;
    if (int r = ring_wait(g, q)) return r;      // the slot's old half may still be landing
    const uint64_t b0 = h * H / kDgenBlock;
    const uint64_t end = (h + 1) * H < g->size ? (h + 1) * H : g->size;
    const uint64_t b1 = (end + kDgenBlock - 1) / kDgenBlock;
    g->held[q] = -1;
    hipStream_t st = g->sg->st[q];
    if (int r = host_launch_blocks(g->sg, dgen_job(g), g->ring->mem + q * H, b0, b1, st)) return r;
    const hipError_t e = hipEventRecord(g->ring->ev[q], st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);
        return s3dg_internal_fail(S3DG_EHIP, (std::string("read-ahead: ") + hipGetErrorString(e)).c_str());
    }
    g->held[q] = (int64_t)h;
    g->pending[q] = true;
    return S3DG_OK;
}

// Return the ring to the pool once nothing is landing in it.
void ring_drop(s3dg_gen *g) {
    if (!g->ring) return;
    for (int q = 0; q < 2; ++q) (void)ring_wait(g, q);
    host_ring_release(g->ring);
    g->ring = nullptr;
    g->held[0] = g->held[1] = -1;
}

// n bytes at the current position through the ring (n < ring half).
int ring_fill(s3dg_gen *g, uint8_t *buf, uint64_t n) {
    if (!g->sg)
        if (int r = host_staging_acquire(g->slot, &g->sg)) return r;
    DeviceScope ds(g->device);
    if (!ds.ok()) return s3dg_internal_fail(S3DG_EHIP, hipGetErrorString(ds.err));
    const uint64_t H = g->ring->half;
    uint64_t done = 0, p = g->pos.load(std::memory_order_relaxed);
    while (done < n) {
        const uint64_t h = p / H;
        if (int r = ring_start(g, h)) return r;
        if (int r = ring_start(g, h + 1)) return r;   // read-ahead
        const int q = (int)(h & 1);
        if (int r = ring_wait(g, q)) return r;
        const uint64_t k = n - done < (h + 1) * H - p ? n - done : (h + 1) * H - p;
        memcpy(buf + done, g->ring->mem + q * H + (p - h * H), k);
        done += k;
        p += k;
    }
    return S3DG_OK;
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
    int device = 0;
    if (int r = s3dg_host_slot_device(slot, &device)) return r;
    s3dg_gen *g = new s3dg_gen();
    g->slot = slot;
    g->device = device;
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
    {
        std::lock_guard<std::mutex> lk(g->mu);
        ring_drop(g);
    }
    host_staging_release(g->sg);
    delete g;
    return S3DG_OK;
}

int s3dg_gen_fill_chunk(s3dg_gen *g, uint8_t *buf, uint64_t cap, uint64_t *written) {
    if (!g || !written) return s3dg_internal_fail(S3DG_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(g->mu);
    *written = 0;
    const uint64_t pos = g->pos.load(std::memory_order_relaxed);
    const uint64_t n = cap < g->size - pos ? cap : g->size - pos;
    if (n == 0) return S3DG_OK;                                     // complete: 0 bytes
    if (!buf) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    const uint64_t H = ring_half();
    if (n < H && !g->ring && !g->ring_none) {
        if (int r = host_ring_acquire(g->slot, H, &g->ring)) return r;
        g->ring_none = g->ring == nullptr;
    }
    if (n < H && g->ring) {
        if (int r = ring_fill(g, buf, n)) return r;
    } else if (int r = fill_range(g, buf, pos, n)) {
        return r;
    }
    g->pos.store(pos + n, std::memory_order_relaxed);
    *written = n;
    if (pos + n == g->size) ring_drop(g);    // complete: the ring goes back to the pool
    return S3DG_OK;
}

int s3dg_gen_fill_at(s3dg_gen *g, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (!g) return s3dg_internal_fail(S3DG_EINVAL, "null generator");
    if (pos > g->size || n > g->size - pos) return s3dg_internal_fail(S3DG_EINVAL, "range past the object");
    std::lock_guard<std::mutex> lk(g->mu);
    return fill_range(g, buf, pos, n);
}

int s3dg_gen_is_complete(s3dg_gen *g) { return g && g->pos.load(std::memory_order_relaxed) >= g->size; }
uint64_t s3dg_gen_position(s3dg_gen *g) { return g ? g->pos.load(std::memory_order_relaxed) : 0; }
uint64_t s3dg_gen_total_size(s3dg_gen *g) { return g ? g->size : 0; }
uint64_t s3dg_gen_seed(s3dg_gen *g) { return g ? g->seed : 0; }
int s3dg_gen_slot(s3dg_gen *g) { return g ? g->slot : -1; }
int s3dg_gen_reset(s3dg_gen *g) {
    if (!g) return s3dg_internal_fail(S3DG_EINVAL, "null generator");
    std::lock_guard<std::mutex> lk(g->mu);
    g->pos.store(0, std::memory_order_relaxed);
    return S3DG_OK;
}

int s3dg_generate_data(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t compress, int has_seed,
                       uint64_t seed) {
    if (size == 0) return S3DG_OK;
    s3dg_gen *g = nullptr;
    if (int r = s3dg_gen_create(size, dedup, compress, has_seed, seed, &g)) return r;
    if (!buf) {
        s3dg_gen_destroy(g);
        return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    }
    int r;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        r = fill_range(g, buf, 0, size);   // one shot: no read-ahead ring
    }
    s3dg_gen_destroy(g);
    return r;
}

}  // extern "C"
