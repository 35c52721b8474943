/*
 * host_stress.c — concurrency stress of the host-buffer drop-ins (host
 * slots, staging sets, the >= 256 MiB split, generators) from many threads,
 * each result checked against the C oracle.  TEST INFRASTRUCTURE: built with
 * the host-ASan/UBSan library by tools/asan_build.sh and run on the GPU box
 * (tools/gpu_r3k.sh); the product tests cover the same calls from Python.
 *
 *   host_stress [threads] [rounds]     prints "STRESS OK" and exits 0
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "s3dlio_gpu.h"

void s3dgo_base_block(uint64_t seed, uint8_t out[4096]);
void s3dgo_fill_controlled(uint8_t *buf, uint64_t len, uint64_t dedup, uint64_t f_num, uint64_t f_den,
                           uint64_t entropy, const uint8_t *base);
void s3dgo_dgen_fill(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t f_num, uint64_t f_den, uint64_t seed);

#define MiB (1024ull * 1024ull)

static uint8_t g_base[4096];
static int g_rounds = 3;
static volatile int g_fail = 0;

static void fail(const char *what, int t, int r) {
    fprintf(stderr, "FAIL thread %d round %d: %s (%s)\n", t, r, what, s3dg_last_error());
    g_fail = 1;
}

static void *worker(void *arg) {
    const int t = (int)(intptr_t)arg;
    for (int r = 0; r < g_rounds && !g_fail; ++r) {
        /* seeded fill_controlled_data of a thread-specific ragged size */
        const uint64_t n = (1 + (t % 5)) * MiB + 4097 * (uint64_t)(t + 1) + (uint64_t)r;
        uint8_t *a = (uint8_t *)malloc(n), *b = (uint8_t *)malloc(n);
        const uint64_t d = 1 + (uint64_t)(t % 4), c = 1 + (uint64_t)(r % 3);
        if (s3dlio_fill_controlled_data_seeded(a, n, d, c, 1000 + t * 10 + r, NULL)) fail("fill seeded", t, r);
        s3dgo_fill_controlled(b, n, d, c > 1 ? c - 1 : 0, c > 1 ? c : 1, 1000 + t * 10 + r, g_base);
        if (memcmp(a, b, n)) fail("fill seeded != oracle", t, r);
        /* generate_data (DG1), seeded */
        if (s3dg_generate_data(a, n, d, c, 1, 77 + t + r)) fail("generate_data", t, r);
        s3dgo_dgen_fill(b, n, d, c > 1 ? c - 1 : 0, c > 1 ? c : 1, 77 + t + r);
        if (memcmp(a, b, n)) fail("generate_data != oracle", t, r);
        /* a generator, filled in uneven chunks */
        s3dg_gen *g = NULL;
        if (s3dg_gen_create(n, d, c, 1, 555 + t, &g) || !g) { fail("gen_create", t, r); free(a); free(b); break; }
        uint64_t pos = 0, w = 0;
        while (!s3dg_gen_is_complete(g)) {
            const uint64_t want = 333333 + 77 * (uint64_t)t;
            const uint64_t cap = n - pos < want ? n - pos : want;
            if (s3dg_gen_fill_chunk(g, a + pos, cap, &w) || w == 0) { fail("gen_fill", t, r); break; }
            pos += w;
        }
        s3dgo_dgen_fill(b, n, d, c > 1 ? c - 1 : 0, c > 1 ? c : 1, 555 + t);
        if (pos != n || memcmp(a, b, n)) fail("generator != oracle", t, r);
        s3dg_gen_destroy(g);
        /* unseeded drop-ins: run, no check beyond success */
        if (s3dlio_fill_controlled_data(a, n, 1, 1) || s3dlio_generate_random_data(a, n)) fail("unseeded", t, r);
        free(a);
        free(b);
    }
    return NULL;
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    g_rounds = argc > 2 ? atoi(argv[2]) : 3;
    s3dgo_base_block(0xBA5EB10C00000000ull, g_base);
    pthread_t th[64];
    for (int t = 0; t < threads && t < 64; ++t) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
    /* meanwhile: one call large enough to split over every slot */
    const uint64_t big = 300 * MiB + 11;
    uint8_t *a = (uint8_t *)malloc(big), *b = (uint8_t *)malloc(big);
    if (s3dlio_fill_controlled_data_seeded(a, big, 2, 3, 4242, NULL)) fail("big split", -1, 0);
    s3dgo_fill_controlled(b, big, 2, 2, 3, 4242, g_base);
    if (memcmp(a, b, big)) fail("big split != oracle", -1, 0);
    free(a);
    free(b);
    for (int t = 0; t < threads && t < 64; ++t) pthread_join(th[t], NULL);
    if (g_fail) return 1;
    printf("STRESS OK\n");
    return 0;
}
