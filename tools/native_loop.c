/* native_loop.c — bench helper, not part of the library: the reference's
 * criterion loop (benches/performance_microbenchmarks.rs:43-64,
 * b.iter(|| fill_controlled_data(&mut buf, dedup, compress))) as a native
 * caller of the C ABI, so bench.py configs 11-13 time the calls the way a
 * Rust caller makes them, without Python's ~2 us per ctypes call.  The entry
 * point is passed in (the library's own s3dg_fill_controlled), so this file
 * links against nothing. */
#include <stdint.h>

typedef int (*fill_fn)(void *ctx, void *dst, uint64_t len, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                       uint64_t entropy, void *stream);

__attribute__((visibility("default"))) int nl_fill_loop(void *fn, void *ctx, void *dst, uint64_t len,
                                                        uint64_t calls, uint64_t dedup, uint32_t f_num,
                                                        uint32_t f_den, uint64_t entropy, void *stream) {
    const fill_fn f = (fill_fn)fn;
    for (uint64_t k = 0; k < calls; ++k) {
        const int r = f(ctx, dst, len, dedup, f_num, f_den, entropy, stream);
        if (r) return r;
    }
    return 0;
}

/* The host-buffer drop-in in the criterion shape: `calls` x
 * s3dlio_fill_controlled_data(buf, len, dedup, compress) on one reused host
 * buffer (benches/performance_microbenchmarks.rs:43-64). */
typedef int (*host_fill_fn)(uint8_t *buf, uint64_t len, uint64_t dedup, uint64_t compress);

__attribute__((visibility("default"))) int nl_host_fill_loop(void *fn, void *buf, uint64_t len, uint64_t calls,
                                                             uint64_t dedup, uint64_t compress) {
    const host_fill_fn f = (host_fill_fn)fn;
    for (uint64_t k = 0; k < calls; ++k) {
        const int r = f((uint8_t *)buf, len, dedup, compress);
        if (r) return r;
    }
    return 0;
}

/* `threads` threads, each making `calls` s3dg_generate_data(buf_t, len, dedup,
 * compress, unseeded) calls into its own buffer: generate_into_buffer from 8
 * Python threads (tests/test_s3dlio_datagen.py:174-204) without the GIL. */
#include <pthread.h>
typedef int (*gen_data_fn)(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t compress, int has_seed,
                           uint64_t seed);
typedef struct {
    gen_data_fn f;
    uint8_t *buf;
    uint64_t len, calls, dedup, compress;
    int rc;
} nl_job;

static void *nl_thread(void *arg) {
    nl_job *J = (nl_job *)arg;
    for (uint64_t k = 0; k < J->calls && !J->rc; ++k) J->rc = J->f(J->buf, J->len, J->dedup, J->compress, 0, 0);
    return 0;
}

__attribute__((visibility("default"))) int nl_threads_gen_loop(void *fn, void **bufs, uint64_t len, int threads,
                                                               uint64_t calls, uint64_t dedup, uint64_t compress) {
    if (threads < 1 || threads > 64) return -1;
    nl_job J[64];
    pthread_t t[64];
    int started = 0, rc = 0;
    for (int q = 0; q < threads; ++q) {
        J[q] = (nl_job){(gen_data_fn)fn, (uint8_t *)bufs[q], len, calls, dedup, compress, 0};
        if (pthread_create(&t[q], 0, nl_thread, &J[q]) != 0) { rc = -2; break; }
        ++started;
    }
    for (int q = 0; q < started; ++q) {
        pthread_join(t[q], 0);
        if (J[q].rc && !rc) rc = J[q].rc;
    }
    return rc;
}

/* ObjectGen::fill_chunk loops (the reference's streaming callers:
 * StreamingDataWriter::generate_remaining 64 KiB, src/streaming_writer.rs:111-116;
 * generate_controlled_data_streaming at Config::chunk_size, src/data_gen.rs:232-249;
 * fill_remaining 32 MiB, :356-367).  nl_gen_collect: one generator's chunks
 * appended into `out` (tests); nl_threads_chunk_loop: `threads` threads, each
 * generating `objs` objects of obj_size bytes chunk by chunk into its own
 * chunk-sized buffer (as fill_chunk's fresh Vec per call), one generator per
 * object, seeded seed_base + thread * objs + k (bench). */
typedef int (*gen_create_fn)(uint64_t size, uint64_t dedup, uint64_t compress, int has_seed, uint64_t seed,
                             void **out);
typedef int (*gen_chunk_fn)(void *g, uint8_t *buf, uint64_t cap, uint64_t *written);
typedef int (*gen_destroy_fn)(void *g);

__attribute__((visibility("default"))) int nl_gen_collect(void *chunk_fn, void *g, uint8_t *out, uint64_t total,
                                                          uint64_t chunk, uint64_t *got) {
    const gen_chunk_fn f = (gen_chunk_fn)chunk_fn;
    uint64_t pos = 0, w = 0;
    *got = 0;
    while (pos < total) {
        const uint64_t cap = total - pos < chunk ? total - pos : chunk;
        const int r = f(g, out + pos, cap, &w);
        if (r) return r;
        if (w == 0) break;
        pos += w;
    }
    *got = pos;
    return 0;
}

typedef struct {
    gen_create_fn create;
    gen_chunk_fn chunk;
    gen_destroy_fn destroy;
    uint8_t *buf;
    uint64_t obj_size, chunk_size, objs, dedup, compress, seed0;
    uint64_t bytes;
    int rc;
} nl_cjob;

static void *nl_chunk_thread(void *arg) {
    nl_cjob *J = (nl_cjob *)arg;
    for (uint64_t k = 0; k < J->objs && !J->rc; ++k) {
        void *g = 0;
        J->rc = J->create(J->obj_size, J->dedup, J->compress, 1, J->seed0 + k, &g);
        if (J->rc) break;
        uint64_t w = 0;
        do {
            J->rc = J->chunk(g, J->buf, J->chunk_size, &w);
            J->bytes += w;
        } while (!J->rc && w);
        J->destroy(g);
    }
    return 0;
}

__attribute__((visibility("default"))) int nl_threads_chunk_loop(void *create_fn, void *chunk_fn, void *destroy_fn,
                                                                 void **bufs, int threads, uint64_t obj_size,
                                                                 uint64_t chunk, uint64_t objs, uint64_t dedup,
                                                                 uint64_t compress, uint64_t seed_base,
                                                                 uint64_t *bytes) {
    if (threads < 1 || threads > 64) return -1;
    nl_cjob J[64];
    pthread_t t[64];
    int started = 0, rc = 0;
    *bytes = 0;
    for (int q = 0; q < threads; ++q) {
        J[q] = (nl_cjob){(gen_create_fn)create_fn, (gen_chunk_fn)chunk_fn, (gen_destroy_fn)destroy_fn,
                         (uint8_t *)bufs[q], obj_size, chunk, objs, dedup, compress,
                         seed_base + (uint64_t)q * objs, 0, 0};
        if (pthread_create(&t[q], 0, nl_chunk_thread, &J[q]) != 0) { rc = -2; break; }
        ++started;
    }
    for (int q = 0; q < started; ++q) {
        pthread_join(t[q], 0);
        if (J[q].rc && !rc) rc = J[q].rc;
        *bytes += J[q].bytes;
    }
    return rc;
}
