/*
 * binding_abi.c — exercises the C ABI exactly as the reference-side Rust
 * binding (integration/rust/src/gpu_data_gen.rs) calls it,
 * one block per reference function, and checks the bytes against the C
 * oracle (oracle/s3dg_oracle.c, linked in) where the layout is seeded.
 * TEST INFRASTRUCTURE: built and run by tests/test_capi_binding.py.
 *
 *   binding_abi <out_dir>      prints "PASS <name>" per check, exit 0 = all pass
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "s3dlio_gpu.h"

/* oracle (test infrastructure) */
void s3dgo_base_block(uint64_t seed, uint8_t out[4096]);
void s3dgo_fill_controlled(uint8_t *buf, uint64_t len, uint64_t dedup, uint64_t f_num, uint64_t f_den,
                           uint64_t entropy, const uint8_t *base);
void s3dgo_dgen_fill(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t f_num, uint64_t f_den, uint64_t seed);

#define MiB (1024ull * 1024ull)
#define CHECK(name, cond)                                                                  \
    do {                                                                                   \
        if (!(cond)) {                                                                     \
            fprintf(stderr, "FAIL %s (line %d): %s\n", name, __LINE__, s3dg_last_error()); \
            return 1;                                                                      \
        }                                                                                  \
        printf("PASS %s\n", name);                                                         \
    } while (0)

static uint8_t *xalloc(uint64_t n) {
    uint8_t *p = (uint8_t *)malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "malloc\n"); exit(2); }
    return p;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const char *dir = argv[1];
    uint8_t base[4096];
    s3dgo_base_block(0xBA5EB10C00000000ull, base);   /* a context's default block */

    /* fill_controlled_data_seeded (src/data_gen.rs:151, seeded sibling) */
    {
        const uint64_t n = 9 * MiB + 4097;
        uint8_t *a = xalloc(n), *b = xalloc(n);
        CHECK("fill_controlled_data_seeded", s3dlio_fill_controlled_data_seeded(a, n, 3, 4, 4242, NULL) == 0);
        s3dgo_fill_controlled(b, n, 3, 3, 4, 4242, base);
        CHECK("fill_controlled_data_seeded == oracle", memcmp(a, b, n) == 0);
        uint8_t user[4096];
        for (int k = 0; k < 4096; ++k) user[k] = (uint8_t)(k * 7 + 1);
        CHECK("fill_controlled_data_seeded(base)", s3dlio_fill_controlled_data_seeded(a, n, 1, 1, 5, user) == 0);
        s3dgo_fill_controlled(b, n, 1, 0, 1, 5, user);
        CHECK("fill_controlled_data_seeded(base) == oracle", memcmp(a, b, n) == 0);
        free(a); free(b);
    }
    /* HostRegistration (register, fill through the guard's slice, drop = unregister) */
    {
        const uint64_t n = 1 * MiB;
        uint8_t *a = xalloc(n), *b = xalloc(n);
        CHECK("HostRegistration::new", s3dg_host_register(a, n) == 0);
        for (int k = 0; k < 3; ++k) {
            CHECK("fill_controlled_data_seeded(registered)",
                  s3dlio_fill_controlled_data_seeded(a, n, 1, 1, 77 + (uint64_t)k, NULL) == 0);
            s3dgo_fill_controlled(b, n, 1, 0, 1, 77 + (uint64_t)k, base);
            CHECK("fill_controlled_data_seeded(registered) == oracle", memcmp(a, b, n) == 0);
        }
        CHECK("HostRegistration drop", s3dg_host_unregister(a) == 1);
        free(a); free(b);   /* after the unregister: the contract */
    }
    /* fill_controlled_data (src/data_gen.rs:151): in place, time entropy */
    {
        const uint64_t n = 2 * MiB;
        uint8_t *a = xalloc(n), *b = xalloc(n);
        CHECK("fill_controlled_data", s3dlio_fill_controlled_data(a, n, 1, 1) == 0 &&
                                          s3dlio_fill_controlled_data(b, n, 1, 1) == 0);
        CHECK("fill_controlled_data: calls differ", memcmp(a, b, n) != 0);
        CHECK("fill_controlled_data: empty is a no-op", s3dlio_fill_controlled_data(NULL, 0, 1, 1) == 0);
        free(a); free(b);
    }
    /* generate_random_data (src/data_gen.rs:102): BASE_BLOCK tiled, windows random */
    {
        const uint64_t n = 3 * 4096 + 100;
        uint8_t *a = xalloc(n);
        CHECK("generate_random_data", s3dlio_generate_random_data(a, n) == 0);
        CHECK("generate_random_data: blocks share the template",
              memcmp(a + 32, a + 4096 + 32, 2048 - 32) == 0 && memcmp(a + 32, a + 8192 + 32, 2048 - 32) == 0);
        CHECK("generate_random_data: windows differ", memcmp(a, a + 4096, 32) != 0);
        free(a);
    }
    /* generate_object (src/data_gen.rs:29): size, then the framed object */
    {
        uint64_t need = 0, w = 0;
        CHECK("object_size(raw)", s3dg_object_size(S3DG_OBJ_RAW, 1, 3 * MiB + 5, &need) == 0 && need == 3 * MiB + 5);
        uint8_t *a = xalloc(need), *b = xalloc(need);
        CHECK("generate_object(raw, controlled, seeded)",
              s3dg_generate_object(S3DG_OBJ_RAW, 1, 3 * MiB + 5, 1, 2, 3, S3DG_MODE_SINGLE_PASS, 1, 77, a, need,
                                   &w) == 0 && w == need);
        s3dgo_dgen_fill(b, need, 2, 2, 3, 77);
        CHECK("generate_object(raw) == DG1 oracle", memcmp(a, b, need) == 0);
        free(a); free(b);
        CHECK("object_size(tfrecord)", s3dg_object_size(S3DG_OBJ_TFRECORD, 4, 1000, &need) == 0 && need == 4 * 1016);
        a = xalloc(need);
        CHECK("generate_object(tfrecord, random)",
              s3dg_generate_object(S3DG_OBJ_TFRECORD, 4, 1000, 0, 1, 1, S3DG_MODE_STREAMING, 0, 0, a, need, &w) == 0 &&
              w == need);
        CHECK("generate_object(hdf5) is an error",
              s3dg_generate_object(S3DG_OBJ_HDF5, 1, 10, 0, 1, 1, 0, 0, 0, a, need, &w) == S3DG_EINVAL);
        free(a);
    }
    /* DataGenerator::begin_object / ObjectGen (src/data_gen.rs:253-371) and
       generate_controlled_data_streaming (:232): chunked, any chunk size */
    {
        const uint64_t n = 5 * MiB + 3, chunk = 777777;
        s3dg_gen *g = NULL;
        CHECK("ObjectGen: create", s3dg_gen_create(n, 4, 2, 1, 99999, &g) == 0 && g);
        CHECK("ObjectGen: total_size", s3dg_gen_total_size(g) == n && s3dg_gen_position(g) == 0);
        uint8_t *a = xalloc(n), *b = xalloc(n);
        uint64_t pos = 0, w = 0;
        while (!s3dg_gen_is_complete(g)) {
            uint64_t cap = n - pos < chunk ? n - pos : chunk;
            if (s3dg_gen_fill_chunk(g, a + pos, cap, &w) != 0 || w == 0) break;
            pos += w;
        }
        CHECK("ObjectGen: exact size", pos == n && s3dg_gen_position(g) == n);
        CHECK("ObjectGen: fill after complete writes 0", s3dg_gen_fill_chunk(g, b, 16, &w) == 0 && w == 0);
        s3dgo_dgen_fill(b, n, 4, 1, 2, 99999);
        CHECK("ObjectGen == DG1 oracle", memcmp(a, b, n) == 0);
        CHECK("ObjectGen: reset", s3dg_gen_reset(g) == 0 && s3dg_gen_position(g) == 0 && !s3dg_gen_is_complete(g));
        CHECK("ObjectGen: fill_remaining", s3dg_gen_fill_chunk(g, b, n, &w) == 0 && w == n && memcmp(a, b, n) == 0);
        CHECK("ObjectGen: seed", s3dg_gen_seed(g) == 99999);
        CHECK("ObjectGen: destroy", s3dg_gen_destroy(g) == 0);
        free(a); free(b);
    }
    /* ObjectGenAlt::new (src/data_gen_alt.rs:95, unseeded) and
       generate_controlled_data_alt (:66) / generate_data (seeded and not) */
    {
        const uint64_t n = 2 * MiB + 9;
        s3dg_gen *g1 = NULL, *g2 = NULL;
        CHECK("ObjectGenAlt::new", s3dg_gen_create(n, 0, 0, 0, 0, &g1) == 0 && s3dg_gen_create(n, 0, 0, 0, 0, &g2) == 0);
        uint8_t *a = xalloc(n), *b = xalloc(n);
        uint64_t w1 = 0, w2 = 0;
        CHECK("ObjectGenAlt::fill_chunk", s3dg_gen_fill_chunk(g1, a, n, &w1) == 0 && s3dg_gen_fill_chunk(g2, b, n, &w2) == 0 &&
                                              w1 == n && w2 == n);
        CHECK("ObjectGenAlt: unseeded instances differ", memcmp(a, b, n) != 0);
        s3dg_gen_destroy(g1); s3dg_gen_destroy(g2);
        CHECK("generate_controlled_data_alt(seed)", s3dg_generate_data(a, n, 3, 2, 1, 4242) == 0);
        s3dgo_dgen_fill(b, n, 3, 1, 2, 4242);
        CHECK("generate_controlled_data_alt == DG1 oracle", memcmp(a, b, n) == 0);
        CHECK("generate_data(None)", s3dg_generate_data(a, n, 1, 1, 0, 0) == 0 && s3dg_generate_data(b, n, 1, 1, 0, 0) == 0 &&
                                         memcmp(a, b, n) != 0);
        free(a); free(b);
    }
    /* dgen surface re-exported by src/data_gen_alt.rs:14-16: generate_data
       (GeneratorConfig, seed honoured), generate_data_simple, DataBuffer */
    {
        const uint64_t n = 3 * MiB + 333;
        uint8_t *a = xalloc(n), *b = xalloc(n), *c = xalloc(n);
        CHECK("dgen generate_data(config{seed})", s3dg_generate_data(a, n, 2, 2, 1, 0xDEADBEEF) == 0 &&
                                                      s3dg_generate_data(b, n, 2, 2, 1, 0xDEADBEEF) == 0);
        CHECK("dgen generate_data: same seed, same bytes", memcmp(a, b, n) == 0);
        s3dgo_dgen_fill(c, n, 2, 1, 2, 0xDEADBEEF);
        CHECK("dgen generate_data == DG1 oracle", memcmp(a, c, n) == 0);
        CHECK("dgen generate_data: other seed differs",
              s3dg_generate_data(b, n, 2, 2, 1, 0x12345678) == 0 && memcmp(a, b, n) != 0);
        CHECK("dgen generate_data_simple", s3dg_generate_data(a, n, 1, 1, 0, 0) == 0 &&
                                               s3dg_generate_data(b, n, 1, 1, 0, 0) == 0 && memcmp(a, b, n) != 0);
        CHECK("dgen generate_data_simple(0 bytes)", s3dg_generate_data(a, 0, 1, 1, 0, 0) == 0);
        free(a); free(b); free(c);
    }
    /* dgen DataGenerator::new(config) with the recommended 32 MiB chunk (the
       PyO3 Generator's default, python_datagen_api.rs:308) */
    {
        const uint64_t n = 40 * MiB + 5, chunk = 32 * MiB;
        s3dg_gen *g = NULL;
        CHECK("dgen DataGenerator::new", s3dg_gen_create(n, 1, 3, 1, 31337, &g) == 0);
        uint8_t *a = xalloc(n), *b = xalloc(n);
        uint64_t w1 = 0, w2 = 0, w3 = 0;
        CHECK("dgen DataGenerator::fill_chunk x2", s3dg_gen_fill_chunk(g, a, chunk, &w1) == 0 && w1 == chunk &&
                                                      s3dg_gen_fill_chunk(g, a + w1, chunk, &w2) == 0 &&
                                                      w2 == n - chunk);
        CHECK("dgen DataGenerator: complete, then 0", s3dg_gen_is_complete(g) && s3dg_gen_fill_chunk(g, b, 8, &w3) == 0 &&
                                                         w3 == 0 && s3dg_gen_position(g) == n);
        s3dgo_dgen_fill(b, n, 1, 2, 3, 31337);
        CHECK("dgen DataGenerator == DG1 oracle", memcmp(a, b, n) == 0);
        s3dg_gen_destroy(g);
        free(a); free(b);
    }
    /* PyO3 generate_into_buffer (python_datagen_api.rs:150): straight into the
       caller's buffer, exactly its bytes (guards around it stay) */
    {
        const uint64_t n = 5 * MiB + 77, pad = 4096;
        uint8_t *a = xalloc(n + 2 * pad);
        memset(a, 0xAB, n + 2 * pad);
        CHECK("PyO3 generate_into_buffer", s3dg_generate_data(a + pad, n, 4, 2, 0, 0) == 0);
        int guards = 1;
        for (uint64_t k = 0; k < pad; ++k) guards &= a[k] == 0xAB && a[pad + n + k] == 0xAB;
        CHECK("PyO3 generate_into_buffer: guards intact", guards);
        uint64_t zeros = 0;
        for (uint64_t k = 0; k < n; ++k) zeros += a[pad + k] == 0;
        CHECK("PyO3 generate_into_buffer: zero fraction ~ (c-1)/c", zeros > n * 45 / 100 && zeros < n * 55 / 100);
        free(a);
    }
    /* PyO3 Generator(size, dedup, compress, threads, chunk_size, seed) and
       generate_data / generate_data_with_threads (python_datagen_api.rs:49-123,
       :270-365): a seeded generator, a buffer larger than what is left */
    {
        const uint64_t n = 2 * MiB + 1;
        s3dg_gen *g = NULL;
        CHECK("PyO3 Generator(seed)", s3dg_gen_create(n, 2, 1, 1, 4242, &g) == 0);
        uint8_t *a = xalloc(4 * MiB), *b = xalloc(n);
        uint64_t w = 0;
        CHECK("PyO3 Generator.fill_chunk(bigger buffer)", s3dg_gen_fill_chunk(g, a, 4 * MiB, &w) == 0 && w == n);
        s3dgo_dgen_fill(b, n, 2, 0, 1, 4242);
        CHECK("PyO3 Generator == DG1 oracle", memcmp(a, b, n) == 0);
        CHECK("PyO3 Generator.is_complete / reset", s3dg_gen_is_complete(g) && s3dg_gen_reset(g) == 0 &&
                                                        !s3dg_gen_is_complete(g));
        s3dg_gen_destroy(g);
        CHECK("PyO3 generate_data", s3dg_generate_data(a, n, 1, 1, 0, 0) == 0);
        CHECK("PyO3 generate_data_with_threads", s3dg_generate_data(b, n, 1, 1, 0, 0) == 0 && memcmp(a, b, n) != 0);
        free(a); free(b);
    }
    /* generate_npz_bytes (python_datagen_api.rs:395) -> generate_npz_bytes_raw (npz.rs:322) */
    {
        s3dg_ctx *ctx = NULL;
        CHECK("host slot context", s3dg_host_slot_context(-1, &ctx) == 0 && ctx);
        const uint64_t shape[3] = {300, 211, 1};
        uint64_t total = 0;
        CHECK("npz_size", s3dg_npz_size(shape, 3, "<f4", 2, &total) == 0 && total > 300 * 211 * 4);
        uint8_t *a = xalloc(total);
        CHECK("npz_build", s3dg_npz_build(ctx, shape, 3, "<f4", 2, a, total) == 0 && a[0] == 'P' && a[1] == 'K');
        char path[4096];
        snprintf(path, sizeof(path), "%s/npz_300x211x1_f4_2.npz", dir);
        FILE *f = fopen(path, "wb");
        CHECK("npz written", f && fwrite(a, 1, total, f) == total);
        fclose(f);
        free(a);
    }
    /* put_objects_with_random_data_and_type (src/s3_utils.rs:1717) on file:// */
    {
        s3dg_ctx *ctx = NULL;
        CHECK("put: slot context", s3dg_host_slot_context(-1, &ctx) == 0);
        char p0[4096], p1[4096], p2[4096];
        snprintf(p0, sizeof(p0), "%s/put/a.bin", dir);
        snprintf(p1, sizeof(p1), "%s/put/b.bin", dir);
        snprintf(p2, sizeof(p2), "%s/put/c.bin", dir);
        const char *paths[3] = {p0, p1, p2};
        uint32_t crc[3] = {0, 0, 0};
        s3dg_put_stats st;
        s3dg_ctx *ctxs[1] = {ctx};
        CHECK("put_objects_multi", s3dg_put_objects_multi(ctxs, 1, paths, 3, MiB + 17, S3DG_OBJ_RAW,
                                                          S3DG_PAYLOAD_CONTROLLED, 2, 1, 2, 5, 4, crc, &st) == 0 &&
                                       st.objects == 3 && st.bytes == 3 * (MiB + 17));
        uint8_t *a = xalloc(MiB + 17), *b = xalloc(MiB + 17);
        FILE *f = fopen(p1, "rb");
        CHECK("put: file written", f && fread(a, 1, MiB + 17, f) == MiB + 17);
        fclose(f);
        s3dgo_fill_controlled(b, MiB + 17, 2, 1, 2, 5 + (1ull << 32), base);
        CHECK("put: object 1 == oracle (entropy seed_base + 2^32)", memcmp(a, b, MiB + 17) == 0);
        CHECK("put: checksum", crc[1] == s3dg_crc32_host(0, b, MiB + 17));
        free(a); free(b);
    }
    /* the pure-host framing the binding re-exports (build_tfrecord / build_npz) */
    {
        uint8_t data[8] = {1, 2, 3, 4, 5, 6, 7, 8}, out[2 * 20], idx[32];
        CHECK("build_tfrecord", s3dg_build_tfrecord(2, 4, data, out, idx) == 0);
        uint64_t nz = 0;
        CHECK("build_npz size", s3dg_npz_legacy_size(8, 8, &nz) == 0 && nz > 8);
    }
    printf("ALL PASS\n");
    return 0;
}
