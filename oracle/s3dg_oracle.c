/*
 * s3dg_oracle.c — CPU restatement of s3dlio's synthetic payload generator.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (s3dlio_amd/, the C-ABI
 * library) links, loads or calls this file.  It is used by tests/ (parity
 * checker), __graft_entry__.smoke() (checker) and bench.py's cpu_baseline
 * leg (timed as kind="port").
 *
 * Parity status:
 *   - PRNG layer (SplitMix64 seeding, Xoshiro256++ next_u64/next_u32,
 *     rand_core 0.9 fill_bytes_via_next) is pinned by the published
 *     known-answer vectors in tests/golden/kat.json.
 *   - Block assembly follows /root/reference/src/data_gen.rs:151-224 line by
 *     line.  The reference cannot be compiled (no Rust toolchain) or imported
 *     (no built _pymod) in this image and it holds no byte-level golden
 *     vectors for this path, so beyond the PRNG KATs the
 *     restatement is cross-checked against an independent Python restatement
 *     (oracle/oracle_py.py) only: "parity unpinned" at the block-assembly
 *     level, pinned at the PRNG level.
 *
 * Entropy injection: the reference draws `call_entropy` from SystemTime
 * (src/data_gen.rs:192-195) and the 4 KiB A_BASE_BLOCK from ThreadRng
 * (src/constants.rs:715-720).  Both are parameters here.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <time.h>

#define S3DGO_BLK 4096u        /* BLK_SIZE   src/constants.rs:326 */
#define S3DGO_HALF 2048u       /* HALF_BLK   src/constants.rs:329 */
#define S3DGO_MOD 32u          /* MOD_SIZE   src/constants.rs:352 */

/* ---- PRNG: rand 0.9.2 SmallRng (64-bit) == Xoshiro256++ ----------------- */

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* SplitMix64 step (seed expansion used by Xoshiro256PlusPlus::seed_from_u64). */
uint64_t s3dgo_splitmix64_next(uint64_t *x) {
    *x += 0x9E3779B97F4A7C15ull;
    uint64_t z = *x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* SmallRng::seed_from_u64 — used at src/data_gen.rs:203 and
 * Xoshiro256PlusPlus::seed_from_u64 at src/data_formats/npz.rs:381. */
void s3dgo_xoshiro_seed(uint64_t s[4], uint64_t seed) {
    uint64_t x = seed;
    for (int k = 0; k < 4; ++k) s[k] = s3dgo_splitmix64_next(&x);
}

uint64_t s3dgo_xoshiro_next(uint64_t s[4]) {
    const uint64_t out = rotl64(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return out;
}

/* rand_core 0.9 le::fill_bytes_via_next: whole u64 words little-endian; a
 * 5..7-byte tail takes the low bytes of one more next_u64; a 1..4-byte tail
 * takes the low bytes of next_u32 == (next_u64 >> 32). */
void s3dgo_fill_bytes(uint64_t s[4], uint8_t *dst, size_t n) {
    size_t off = 0;
    for (; n - off >= 8; off += 8) {
        uint64_t w = s3dgo_xoshiro_next(s);
        for (int b = 0; b < 8; ++b) dst[off + b] = (uint8_t)(w >> (8 * b));
    }
    size_t tail = n - off;
    if (tail > 4) {
        uint64_t w = s3dgo_xoshiro_next(s);
        for (size_t b = 0; b < tail; ++b) dst[off + b] = (uint8_t)(w >> (8 * b));
    } else if (tail > 0) {
        uint32_t w = (uint32_t)(s3dgo_xoshiro_next(s) >> 32);
        for (size_t b = 0; b < tail; ++b) dst[off + b] = (uint8_t)(w >> (8 * b));
    }
}

/* The build-defined deterministic base block (stands in for A_BASE_BLOCK,
 * src/constants.rs:715-720): Xoshiro256++ seeded from `seed`, 4096 bytes. */
void s3dgo_base_block(uint64_t seed, uint8_t out[S3DGO_BLK]) {
    uint64_t s[4];
    s3dgo_xoshiro_seed(s, seed);
    s3dgo_fill_bytes(s, out, S3DGO_BLK);
}

/* ---- fill_controlled_data (src/data_gen.rs:151-224) ---------------------- */

/* unique_blocks, src/data_gen.rs:162-167 (f64 division, round half away). */
uint64_t s3dgo_unique_blocks(uint64_t nblocks, uint64_t dedup) {
    uint64_t d = dedup == 0 ? 1 : dedup;
    if (d <= 1) return nblocks;
    double r = round((double)nblocks / (double)d);
    if (r < 1.0) r = 1.0;
    return (uint64_t)r;
}

/* compress -> (f_num, f_den), src/data_gen.rs:169-173. */
void s3dgo_compress_ratio(uint64_t compress, uint64_t *f_num, uint64_t *f_den) {
    if (compress > 1) { *f_num = compress - 1; *f_den = compress; }
    else { *f_num = 0; *f_den = 1; }
}

/* Per-unique-block zero-prefix lengths by the reference's Bresenham
 * accumulator (src/data_gen.rs:174-190).  Caller frees. */
static uint64_t *const_len_table(uint64_t unique, uint64_t f_num, uint64_t f_den) {
    uint64_t *v = (uint64_t *)malloc(sizeof(uint64_t) * (unique ? unique : 1));
    const uint64_t floor_len = (f_num * S3DGO_BLK) / f_den;
    const uint64_t rem = (f_num * S3DGO_BLK) % f_den;
    uint64_t acc = 0;
    for (uint64_t k = 0; k < unique; ++k) {
        acc += rem;
        if (acc >= f_den) { acc -= f_den; v[k] = floor_len + 1; }
        else v[k] = floor_len;
    }
    return v;
}

/* One 4 KiB block (body of the par_chunks_mut closure, :200-222). */
static void fill_one_block(uint8_t *chunk, uint64_t len, uint64_t i, uint64_t unique,
                           const uint64_t *const_lens, uint64_t entropy,
                           const uint8_t *base) {
    const uint64_t u = i % unique;
    uint64_t s[4];
    s3dgo_xoshiro_seed(s, u + entropy);                 /* wrapping add, :202 */
    memcpy(chunk, base, len);                           /* :205-207 */
    uint64_t c = const_lens[u] < len ? const_lens[u] : len;
    memset(chunk, 0, c);                                /* :209-210 */
    uint64_t region = len - c;
    uint64_t m = region < S3DGO_MOD ? region : S3DGO_MOD;
    if (m > 0) {
        s3dgo_fill_bytes(s, chunk + c, m);              /* :217 */
        uint64_t so = c > S3DGO_HALF ? c : S3DGO_HALF;  /* :218 */
        if (so + m <= len) s3dgo_fill_bytes(s, chunk + so, m);   /* :219-221 */
    }
}

void s3dgo_fill_controlled(uint8_t *buf, uint64_t len, uint64_t dedup,
                           uint64_t f_num, uint64_t f_den, uint64_t entropy,
                           const uint8_t *base) {
    if (len == 0) return;                               /* :154-156 */
    const uint64_t nblocks = (len + S3DGO_BLK - 1) / S3DGO_BLK;
    const uint64_t unique = s3dgo_unique_blocks(nblocks, dedup);
    uint64_t *cl = const_len_table(unique, f_num, f_den);
    for (uint64_t i = 0; i < nblocks; ++i) {
        uint64_t off = i * S3DGO_BLK;
        uint64_t l = len - off < S3DGO_BLK ? len - off : S3DGO_BLK;
        fill_one_block(buf + off, l, i, unique, cl, entropy, base);
    }
    free(cl);
}

/* Build-defined per-object entropy:
 * object j of a stream gets E_j = seed_base + j * 2^32, so that the
 * reference's `u + E` seeds (u < 2^32) never alias across objects. */
uint64_t s3dgo_object_entropy(uint64_t seed_base, uint64_t j) {
    return seed_base + (j << 32);
}

/* A stream of n equal-size objects at a fixed stride (single-threaded). */
void s3dgo_fill_stream(uint8_t *dst, uint64_t obj_size, uint64_t stride, uint64_t n,
                       uint64_t dedup, uint64_t f_num, uint64_t f_den,
                       uint64_t seed_base, uint64_t first_obj, const uint8_t *base) {
    for (uint64_t j = 0; j < n; ++j)
        s3dgo_fill_controlled(dst + j * stride, obj_size, dedup, f_num, f_den,
                              s3dgo_object_entropy(seed_base, first_obj + j), base);
}

/* ---- multi-threaded form: the CPU baseline ------------------------------- */
/* Mirrors the reference's Rayon par_chunks_mut(4096) over every block of the
 * object (src/data_gen.rs:198): a pool of `threads` workers pulls runs of
 * blocks from one atomic counter (dynamic load balance, like work stealing). */

typedef struct {
    uint8_t *dst; uint64_t obj_size, stride, n, nblocks, unique;
    const uint64_t *cl; uint64_t seed_base, first_obj; const uint8_t *base;
    _Atomic uint64_t next; uint64_t total, grain;
} mt_job;

#define MT_GRAIN 64u

static void *mt_worker(void *arg) {
    mt_job *J = (mt_job *)arg;
    const uint64_t grain = J->grain ? J->grain : MT_GRAIN;
    for (;;) {
        uint64_t g0 = atomic_fetch_add(&J->next, grain);
        if (g0 >= J->total) break;
        uint64_t g1 = g0 + grain < J->total ? g0 + grain : J->total;
        for (uint64_t g = g0; g < g1; ++g) {
            uint64_t j = g / J->nblocks, i = g % J->nblocks;
            uint64_t off = i * S3DGO_BLK;
            uint64_t l = J->obj_size - off < S3DGO_BLK ? J->obj_size - off : S3DGO_BLK;
            fill_one_block(J->dst + j * J->stride + off, l, i, J->unique, J->cl,
                           s3dgo_object_entropy(J->seed_base, J->first_obj + j), J->base);
        }
    }
    return NULL;
}

int s3dgo_fill_stream_mt(uint8_t *dst, uint64_t obj_size, uint64_t stride, uint64_t n,
                         uint64_t dedup, uint64_t f_num, uint64_t f_den,
                         uint64_t seed_base, uint64_t first_obj, const uint8_t *base,
                         int threads) {
    if (obj_size == 0 || n == 0) return 0;
    if (threads < 1) threads = 1;
    mt_job J;
    J.dst = dst; J.obj_size = obj_size; J.stride = stride; J.n = n;
    J.nblocks = (obj_size + S3DGO_BLK - 1) / S3DGO_BLK;
    J.unique = s3dgo_unique_blocks(J.nblocks, dedup);
    uint64_t *cl = const_len_table(J.unique, f_num, f_den);
    J.cl = cl; J.seed_base = seed_base; J.first_obj = first_obj; J.base = base;
    atomic_init(&J.next, 0);
    J.total = J.nblocks * n;
    J.grain = MT_GRAIN;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    int started = 0;
    for (int t = 1; t < threads; ++t)
        if (pthread_create(&tid[started], NULL, mt_worker, &J) == 0) ++started;
    mt_worker(&J);                      /* the calling thread works too */
    for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
    free(tid);
    free(cl);
    return started + 1;
}

/* ---- persistent pool: the reference's criterion shape --------------------- */
/* benches/performance_microbenchmarks.rs:43-64 calls fill_controlled_data on
 * one reused 1/4/16 MiB Vec in a loop, on Rayon's global pool, which lives for
 * the process.  Creating threads per call (s3dgo_fill_stream_mt) would charge
 * each 1 MiB call tens of microseconds of pthread_create, so this form keeps
 * `threads - 1` workers parked on a condition variable; the calling thread
 * works too.  Blocks go out in grains of total / (8 * threads) (1..64), close
 * to Rayon's adaptive splitting of par_chunks_mut. */
static struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int workers;
    int helpers;            /* workers 0 .. helpers-1 take part in the current job */
    _Atomic uint64_t gen;
    mt_job *job;
    _Atomic int busy;
} g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0, NULL, 0};

static void *pool_worker(void *arg) {
    const int id = (int)(intptr_t)arg;
    uint64_t seen = 0;
    for (;;) {
        /* spin a while before parking, as Rayon's workers do, so back-to-back
           calls do not pay a futex wake each */
        for (int k = 0; k < 200000 && atomic_load_explicit(&g_pool.gen, memory_order_acquire) == seen; ++k)
            __builtin_ia32_pause();
        pthread_mutex_lock(&g_pool.mu);
        while (atomic_load(&g_pool.gen) == seen) pthread_cond_wait(&g_pool.cv, &g_pool.mu);
        seen = atomic_load(&g_pool.gen);
        mt_job *J = g_pool.job;
        const int part = id < g_pool.helpers;
        pthread_mutex_unlock(&g_pool.mu);
        if (part) mt_worker(J);
        atomic_fetch_sub(&g_pool.busy, 1);
    }
    return NULL;
}

/* One fill_controlled_data call on `buf` (seeded by `entropy`) over the pool;
 * not reentrant (one caller at a time).  Returns the threads used. */
int s3dgo_pool_fill_controlled(uint8_t *buf, uint64_t len, uint64_t dedup, uint64_t f_num,
                               uint64_t f_den, uint64_t entropy, const uint8_t *base, int threads) {
    if (len == 0) return 0;
    if (threads < 1) threads = 1;
    pthread_mutex_lock(&g_pool.mu);
    while (g_pool.workers < threads - 1) {
        pthread_t t;
        if (pthread_create(&t, NULL, pool_worker, (void *)(intptr_t)g_pool.workers) != 0) break;
        pthread_detach(t);
        ++g_pool.workers;
    }
    const int helpers = g_pool.workers < threads - 1 ? g_pool.workers : threads - 1;
    pthread_mutex_unlock(&g_pool.mu);
    mt_job J;
    J.dst = buf; J.obj_size = len; J.stride = len; J.n = 1;
    J.nblocks = (len + S3DGO_BLK - 1) / S3DGO_BLK;
    J.unique = s3dgo_unique_blocks(J.nblocks, dedup);
    uint64_t *cl = const_len_table(J.unique, f_num, f_den);
    J.cl = cl; J.seed_base = entropy; J.first_obj = 0; J.base = base;
    atomic_init(&J.next, 0);
    J.total = J.nblocks;
    uint64_t grain = J.total / (8u * (uint64_t)threads);
    J.grain = grain < 1 ? 1 : (grain > MT_GRAIN ? MT_GRAIN : grain);
    /* every parked worker wakes and checks in; only the first `helpers` work */
    pthread_mutex_lock(&g_pool.mu);
    g_pool.helpers = helpers;
    atomic_store(&g_pool.busy, g_pool.workers);
    g_pool.job = &J;
    atomic_fetch_add_explicit(&g_pool.gen, 1, memory_order_release);
    pthread_cond_broadcast(&g_pool.cv);
    pthread_mutex_unlock(&g_pool.mu);
    mt_worker(&J);
    while (atomic_load(&g_pool.busy) > 0) { }
    free(cl);
    return helpers + 1;
}

/* ---- generate_npz_bytes_raw x-fill (src/data_formats/npz.rs:376-383) ----- */
/* Chunk k of `chunk` bytes (last one ragged) is filled by
 * Xoshiro256PlusPlus::seed_from_u64(seed_base + k).fill_bytes(chunk). */
void s3dgo_xoshiro_chunks(uint8_t *buf, uint64_t len, uint64_t chunk, uint64_t seed_base) {
    for (uint64_t k = 0, off = 0; off < len; ++k, off += chunk) {
        uint64_t n = len - off < chunk ? len - off : chunk;
        uint64_t s[4];
        s3dgo_xoshiro_seed(s, seed_base + k);
        s3dgo_fill_bytes(s, buf + off, n);
    }
}

/* ---- DG1: the build-defined dgen-contract layout --------- */
/* Parity unpinned (dgen-data 0.2.4 is absent): this restates the build's own
 * definition so the kernel is checked against an independent CPU version.
 * 1 MiB blocks (DGEN_BLOCK_SIZE, src/constants.rs:348); block i =
 * Xoshiro256++ seed_from_u64(seed ^ ((i % U) * phi)).fill_bytes(L), first
 * floor(L * f_num / f_den) bytes zero; U as src/data_gen.rs:162-167. */
void s3dgo_dgen_fill(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t f_num,
                     uint64_t f_den, uint64_t seed) {
    const uint64_t B = 1ull << 20;
    const uint64_t nb = (size + B - 1) / B;
    const uint64_t U = s3dgo_unique_blocks(nb, dedup == 0 ? 1 : dedup);
    for (uint64_t i = 0; i < nb; ++i) {
        const uint64_t off = i * B, L = size - off < B ? size - off : B;
        uint64_t s[4];
        s3dgo_xoshiro_seed(s, seed ^ ((i % U) * 0x9E3779B97F4A7C15ull));
        s3dgo_fill_bytes(s, buf + off, L);
        memset(buf + off, 0, (L * f_num) / f_den);
    }
}

/* ---- seeded analogue of generate_random_data (src/data_gen.rs:102-132) ---- */
/* Reference: BASE_BLOCK tiled per 4 KiB block (:104-107), then one
 * sequential ThreadRng fills [0, min(32, bs)) (:115-122) and, when
 * bs > HALF_BLK, [bs-32, bs) (:124-126) of every block.  ThreadRng is
 * unseedable, so the build seeds each block separately: block i uses
 * SmallRng::seed_from_u64(entropy + i) for both fills (parity impossible,
 * structure identical). */
void s3dgo_random_data(uint8_t *buf, uint64_t size, uint64_t entropy, const uint8_t *base) {
    for (uint64_t off = 0, i = 0; off < size; off += S3DGO_BLK, ++i) {
        uint64_t bs = size - off < S3DGO_BLK ? size - off : S3DGO_BLK;
        memcpy(buf + off, base, bs);
        uint64_t s[4];
        s3dgo_xoshiro_seed(s, entropy + i);
        s3dgo_fill_bytes(s, buf + off, bs < S3DGO_MOD ? bs : S3DGO_MOD);
        if (bs > S3DGO_HALF) s3dgo_fill_bytes(s, buf + off + bs - S3DGO_MOD, S3DGO_MOD);
    }
}

/* ---- DG1 chunked streaming on the CPU (the CPU baseline of bench.py's
 * fill_chunk configs; test infrastructure) ----------------------------------
 * The same bytes as s3dgo_dgen_fill, produced chunk by chunk the way a CPU
 * ObjectGen::fill_chunk caller sees them (src/data_gen.rs:327-336 over
 * ObjectGenAlt, src/data_gen_alt.rs:89-149): the current block's PRNG state
 * and its last drawn word carry over between chunks, so no byte is drawn
 * twice.  Positions only move forward (a backward position reseeds). */
typedef struct {
    uint64_t size, f_num, f_den, seed, U, pos;
    uint64_t s[4];
    uint64_t blk;       /* block whose state is in s (UINT64_MAX: none) */
    uint64_t wnext;     /* index of the next word s yields within the block */
    uint64_t word;      /* word wnext - 1, as fill_bytes_via_next stores it */
} s3dgo_dgen_stream;

void s3dgo_dgen_stream_init(s3dgo_dgen_stream *g, uint64_t size, uint64_t dedup, uint64_t f_num,
                            uint64_t f_den, uint64_t seed) {
    const uint64_t B = 1ull << 20;
    g->size = size; g->f_num = f_num; g->f_den = f_den; g->seed = seed; g->pos = 0;
    g->U = s3dgo_unique_blocks((size + B - 1) / B, dedup == 0 ? 1 : dedup);
    g->blk = UINT64_MAX; g->wnext = 0; g->word = 0;
}

/* word wi of the current block (len L): the last partial word follows the
 * 1..4-byte next_u32 rule of s3dgo_fill_bytes. */
static inline uint64_t dgen_stream_word(s3dgo_dgen_stream *g, uint64_t wi, uint64_t L) {
    while (g->wnext <= wi) {
        uint64_t w = s3dgo_xoshiro_next(g->s);
        const uint64_t tail = L - 8 * g->wnext;
        if (tail < 8 && tail <= 4) w >>= 32;
        g->word = w;
        ++g->wnext;
    }
    return g->word;
}

uint64_t s3dgo_dgen_stream_fill(s3dgo_dgen_stream *g, uint8_t *dst, uint64_t cap) {
    const uint64_t B = 1ull << 20;
    uint64_t n = g->size - g->pos < cap ? g->size - g->pos : cap, done = 0;
    while (done < n) {
        const uint64_t i = g->pos / B, off = i * B, L = g->size - off < B ? g->size - off : B;
        uint64_t o = g->pos - off;
        if (g->blk != i || g->wnext > o / 8 + 1) {
            s3dgo_xoshiro_seed(g->s, g->seed ^ ((i % g->U) * 0x9E3779B97F4A7C15ull));
            g->blk = i; g->wnext = 0;
        }
        const uint64_t end = L < o + (n - done) ? L : o + (n - done);
        uint8_t *d = dst + done;
        const uint64_t o0 = o;
        while (o < end && (o & 7)) { *d++ = (uint8_t)(dgen_stream_word(g, o / 8, L) >> (8 * (o & 7))); ++o; }
        while (o + 8 <= end && 8 * g->wnext == o && o + 8 <= L) {   /* whole words, straight from the PRNG */
            const uint64_t w = s3dgo_xoshiro_next(g->s);
            memcpy(d, &w, 8);
            g->word = w; ++g->wnext; d += 8; o += 8;
        }
        while (o < end) { *d++ = (uint8_t)(dgen_stream_word(g, o / 8, L) >> (8 * (o & 7))); ++o; }
        const uint64_t z = (L * g->f_num) / g->f_den;     /* zero prefix of the block */
        if (o0 < z) memset(dst + done, 0, (z < end ? z : end) - o0);
        done += end - o0;
        g->pos += end - o0;
    }
    return n;
}

/* `threads` threads, each generating objects of obj_size bytes chunk by chunk
 * into its own chunk-sized buffer until `seconds` have passed; object k of
 * thread t seeded seed_base + t * 1000003 + k.  Returns the bytes made. */
typedef struct {
    uint64_t obj_size, chunk, dedup, f_num, f_den, seed0;
    double seconds;
    uint64_t bytes;
} chunk_bench_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *chunk_bench_worker(void *arg) {
    chunk_bench_job *J = (chunk_bench_job *)arg;
    uint8_t *buf = (uint8_t *)malloc(J->chunk);
    memset(buf, 1, J->chunk);
    const double t0 = now_s();
    for (uint64_t k = 0; now_s() - t0 < J->seconds; ++k) {
        s3dgo_dgen_stream g;
        s3dgo_dgen_stream_init(&g, J->obj_size, J->dedup, J->f_num, J->f_den, J->seed0 + k);
        uint64_t w;
        while ((w = s3dgo_dgen_stream_fill(&g, buf, J->chunk)) > 0) J->bytes += w;
    }
    free(buf);
    return NULL;
}

uint64_t s3dgo_dgen_chunk_bench(int threads, uint64_t obj_size, uint64_t chunk, uint64_t dedup, uint64_t f_num,
                                uint64_t f_den, uint64_t seed_base, double seconds, double *elapsed) {
    if (threads < 1) threads = 1;
    chunk_bench_job *J = (chunk_bench_job *)calloc((size_t)threads, sizeof(chunk_bench_job));
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    const double t0 = now_s();
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        J[t] = (chunk_bench_job){obj_size, chunk, dedup, f_num, f_den, seed_base + (uint64_t)t * 1000003ull, seconds, 0};
        if (pthread_create(&tid[started], NULL, chunk_bench_worker, &J[t]) == 0) ++started;
    }
    uint64_t bytes = 0;
    for (int t = 0; t < started; ++t) {
        pthread_join(tid[t], NULL);
        bytes += J[t].bytes;
    }
    *elapsed = now_s() - t0;
    free(J);
    free(tid);
    return bytes;
}
