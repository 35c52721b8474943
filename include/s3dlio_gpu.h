/*
 * s3dlio_gpu.h — C ABI of the MI355X-native synthetic object-payload
 * generator (drop-in for s3dlio's src/data_gen.rs hot path).
 *
 * Every entry point is plain C: pointers, sizes, integers.  All functions
 * return 0 on success or a negative S3DG_E* code; s3dg_last_error() returns
 * a thread-local message for the last failure on the calling thread.
 *
 * Reference interfaces replaced (paths relative to the s3dlio checkout):
 *   s3dlio_fill_controlled_data         src/data_gen.rs:151  fill_controlled_data(buf,dedup,compress)
 *   s3dlio_fill_controlled_data_seeded  src/data_gen.rs:151  (seeded sibling)
 *   s3dg_fill_controlled                src/data_gen.rs:198-223 (the Rayon par_chunks_mut loop)
 *   s3dg_fill_controlled_stream         src/s3_utils.rs:1741 / src/bin/cli.rs:2282 generate_object
 *                                       fan-out, one payload per object
 *   s3dg_fill_controlled_batch          same, mixed object sizes (BASELINE config 4)
 *   s3dg_unique_blocks                  src/data_gen.rs:162-167
 *   s3dg_compress_ratio                 src/data_gen.rs:169-173
 *
 * Device pointers passed to s3dg_fill_* must be 16-byte aligned (objects in
 * a stream/batch too); `stream` is a hipStream_t (NULL = legacy default).
 */
#ifndef S3DLIO_GPU_H
#define S3DLIO_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#pragma GCC visibility push(default)

#define S3DG_BLOCK_SIZE 4096u   /* BLK_SIZE, src/constants.rs:326 */

enum {
    S3DG_OK = 0,
    S3DG_EINVAL = -1,   /* bad argument (null, misaligned, out of range) */
    S3DG_EHIP = -2,     /* HIP runtime error (message in s3dg_last_error) */
    S3DG_ENOMEM = -3,
    S3DG_EIO = -4,      /* file-system error in the put pipeline */
};

typedef struct s3dg_ctx s3dg_ctx;

/* One object of a batch: `dst_off` bytes from dst_base (multiple of 16),
 * `size` bytes, block seeds `u + entropy` (src/data_gen.rs:202), zero-prefix
 * ratio f_num/f_den of each 4 KiB block (compress c -> (c-1, c)). */
typedef struct {
    uint64_t dst_off;
    uint64_t size;
    uint64_t entropy;
    uint64_t dedup;
    uint32_t f_num;
    uint32_t f_den;
} s3dg_obj_desc;

/* ---- context ------------------------------------------------------------ */
int s3dg_ctx_create(int device, s3dg_ctx **out);
int s3dg_ctx_destroy(s3dg_ctx *ctx);
int s3dg_ctx_device(s3dg_ctx *ctx, int *device);
/* Replace the 4 KiB base block (stands in for A_BASE_BLOCK,
 * src/constants.rs:715-720).  Host pointer, 4096 bytes. */
int s3dg_set_base_block(s3dg_ctx *ctx, const uint8_t *base4096);
/* Base block = Xoshiro256++(seed_from_u64(seed)).fill_bytes(4096). */
int s3dg_set_base_block_seed(s3dg_ctx *ctx, uint64_t seed);
int s3dg_get_base_block(s3dg_ctx *ctx, uint8_t *out4096);
/* Wave64s per 4 KiB block = workgroup size / 64: 1, 2 or 4; 0 = auto
 * (2 for streams, 1 for batches).  A tuning knob; results are identical. */
int s3dg_set_waves_per_block(s3dg_ctx *ctx, int waves);
/* 1 = nontemporal stores in every fill kernel, 0 = the default policies. */
int s3dg_set_nontemporal(s3dg_ctx *ctx, int on);
/* Cache policy of the fill kernels' 16-byte stores, for stream and batch
 * launches: 0 = plain, 1 = nt, 2 = sc1, 3 = nt sc1, negative = default
 * (nt sc1 for streams; sc1 for tiled batch launches and nt sc1 for batch
 * launches in the dense layout, measured on MI355X).  A non-negative batch
 * policy applies to both batch layouts.  Results are identical. */
int s3dg_set_store_policy(s3dg_ctx *ctx, int stream_policy, int batch_policy);
/* Cap on resident fill workgroups per CU (reserved LDS), for stream and
 * batch launches separately; 0 = hardware maximum, negative = the default.
 * Defaults, measured on MI355X: 14 (stream); batch launches (and large
 * uniform streams, which run through the batch kernel) per launch: no cap,
 * or 29 resident when most of the launch's blocks have a zero prefix ending on
 * a 64-B line (64 f_num / f_den whole: compress 2, 4, 8, ...).  A cap of k
 * reserves the LDS that leaves floor(160 KiB / footprint) resident, which the
 * 512-B allocation granule can make k - 1 (30 gives 29); s3dg_query_occupancy
 * reports the resident count.  A tuning knob; results are identical. */
int s3dg_set_occupancy(s3dg_ctx *ctx, int stream_wgs_per_cu, int batch_wgs_per_cu);
/* Batch kernel (batches and large uniform streams): the stores of each 4 KiB
 * block wait until `ticks` wall-clock ticks (10 ns) after its workgroup
 * started; 0 = no floor, negative = per launch (100 when most of the
 * launch's blocks have a zero prefix of at least half the block that ends
 * inside a 64-B line, e.g. compress 3, and for uniform streams of objects of
 * >= 2 MiB without a zero prefix; none otherwise).  Measured on MI355X;
 * results are identical. */
int s3dg_set_batch_pace(s3dg_ctx *ctx, int ticks);
/* Batch launches: distance (in units of 64 blocks) at which workgroups warm
 * the L2 with later tile records; 0 = off, UINT32_MAX = default (256).
 * Results are identical. */
int s3dg_set_batch_prefetch(s3dg_ctx *ctx, uint32_t tiles);
/* Batch launches: blocks per tile record (2, 4, 8, 16, 32 or 64), 1 = dense (one
 * record per 4 KiB granule of the batch's address range; used only when
 * the objects are 4 KiB-aligned, sorted and non-overlapping); 0 = chosen per
 * sub-batch by cost (default).  Results are identical. */
int s3dg_set_batch_tile(s3dg_ctx *ctx, uint32_t blocks);
/* Batch launches with per-launch tile sizes: objects of fewer than `blocks`
 * 4 KiB blocks go to a launch of their own (each class with the tile size
 * that suits it), so small objects do not pad large tiles with dead slots;
 * 0 = one launch, negative = default.  Results are identical. */
int s3dg_set_batch_split(s3dg_ctx *ctx, int blocks);
/* 1 = run large uniform streams (>= 64 MiB, objects 32 KiB-aligned relative
 * to each other) through the tiled batch kernel with device-built tile
 * records and the batch launch knobs; 0 = always the 2D stream kernel;
 * negative = default (1).  Results are identical. */
int s3dg_set_stream_tiles(s3dg_ctx *ctx, int on);
/* Keystream kernel launch shape for mode 0 (npz keystream, s3dg_xoshiro_fill)
 * or mode 1 (DG1, s3dg_dgen_fill and the generators): draws staged per lane
 * per store round (16, 32 or 64), waves per workgroup (1, 2 or 4), resident
 * workgroups per CU cap (0 = none), draws per lane (>= 64; sets lanes per
 * chunk; launches too small to fill the GPU use shorter spans, down to 256), store cache policy (as s3dg_set_store_policy, negative =
 * default).  0 = default for each (both modes: 64, 1, 2048 draws, sc1; K2
 * launches of >= 4 rounds of resident waves: 4096 draws; DG1 with a zero
 * prefix: 4 waves, 512 draws).
 * A tuning knob; results are identical. */
int s3dg_set_keystream_shape(s3dg_ctx *ctx, int mode, int draws, int waves, int wgs_per_cu,
                             uint64_t min_lane_draws, int store_policy);
/* Keystream launches (mode 0 / 1): workgroups are remapped so each XCD
 * writes runs of `waves` adjacent waves' lane regions (power of two; at or
 * below the waves per workgroup = the dispatcher's round-robin order; 0 =
 * default: 16, DG1 with a zero prefix 32).  A tuning knob; results are
 * identical. */
int s3dg_set_keystream_xcd_group(s3dg_ctx *ctx, int mode, uint32_t waves);
/* Keystream launches (both modes) of at least `rounds` rounds of resident
 * waves run a persistent grid: one round of workgroups whose waves take work
 * units from per-XCD queues (an XCD that runs ahead takes over units of a
 * slower one instead of idling at the end of the launch).  0 = never; negative
 * = default: 1-wave workgroups from 6 rounds.  A tuning knob; results are
 * identical. */
int s3dg_set_keystream_persist(s3dg_ctx *ctx, int rounds);
/* DG1 launches with a zero prefix (compress > 1) of at least `chunks` whole
 * 1 MiB blocks (all of them full length) run as two launches: the blocks'
 * zero prefixes in the fill's store shape (whole 4 KiB granules, every XCD on
 * every 8th), then the keystream over the blocks' tails only.  chunks: 0 =
 * always one keystream launch, negative = default (64).  The zero launch:
 * `waves` per 4 KiB workgroup (1, 2, 4), `occupancy` resident workgroups per
 * CU cap (0 = none), `store` policy (as s3dg_set_store_policy), `overlap` 1 =
 * on a side stream concurrent with the tails (the caller's stream waits for
 * both); negative = default for each (measured per prefix class: prefixes
 * ending on a 64-B line, e.g. compress 2 or 4: 4 waves, 5 per CU, nt sc1, in
 * order; others: 1 wave, 14 per CU, nt sc1, overlapped).  A tuning knob;
 * results are identical. */
int s3dg_set_dgen_zero_split(s3dg_ctx *ctx, int chunks, int waves, int occupancy, int store, int overlap);
/* One-object DG1 launches that run a persistent grid (see above): their last
 * `chunks` 1 MiB blocks in lanes of half the length, handed out after the
 * others, so the launch drains on shorter units.  0 = off; negative =
 * default (half a resident round of units).  A tuning knob; results are
 * identical. */
int s3dg_set_keystream_tail(s3dg_ctx *ctx, int chunks);
int s3dg_query_keystream_occupancy(s3dg_ctx *ctx, int mode, int *wgs_per_cu);
/* Resident workgroups per CU the current settings give (HIP occupancy API):
 * batch 0 = stream launches, 1 = batch launches, 2 = batch launches whose
 * zero prefixes end on a 64-B line (see s3dg_set_occupancy). */
int s3dg_query_occupancy(s3dg_ctx *ctx, int batch, int *wgs_per_cu);

/* ---- parameter helpers (host math shared with the kernels) --------------- */
uint64_t s3dg_unique_blocks(uint64_t nblocks, uint64_t dedup);
int s3dg_compress_ratio(uint64_t compress, uint32_t *f_num, uint32_t *f_den);
/* Launch class of compress (f_num, f_den) for the batch kernel's per-launch
 * settings: 1 = zero prefix ending on a 64-B line (occupancy
 * cap: 29 resident workgroups per CU, which s3dg_query_occupancy(ctx, 2, ..)
 * reports; the 512-B LDS granule admits no footprint giving exactly 30),
 * 2 = zero prefix of at least half the block ending inside a line (store
 * floor 100 ticks), 0 = otherwise, or f_den = 0 (no cap, no floor). */
int s3dg_zero_class(uint32_t f_num, uint32_t f_den);
/* Batch-kernel launches of zero class 2 (above) check their store floor by
 * measurement: the context times its own launches of >= 1 GiB and runs the
 * floor or a plain launch (the means of each one's last five rates, after
 * four launches of each, the context's first timed launch not counted; the
 * other is taken only when more than 1 % faster than the current choice, so
 * near-equal candidates do not flip between runs), re-probing the other after
 * 32 launches, an interval that doubles with every probe that confirms the
 * choice (up to 1024); class 1 keeps its cap.  An explicit
 * s3dg_set_occupancy / s3dg_set_batch_pace (or env S3DG_ZC_TUNE=0) turns this
 * off.  Query (zclass 0-2): the choice (0 = the class setting, 1 = plain),
 * each one's mean recent GB/s (0 = not measured yet) and the timed launch
 * count.  Results are identical. */
int s3dg_query_zero_tune(s3dg_ctx *ctx, int zclass, int *best, double *rule_gbs, double *plain_gbs,
                         uint64_t *timed);
/* Per-object entropy of object j of a stream: seed_base + j * 2^32. */
uint64_t s3dg_object_entropy(uint64_t seed_base, uint64_t j);

/* ---- device-resident generation (asynchronous on `stream`) -------------- */
/* One object of `len` bytes at dst (device).  From 64 MiB up this runs as a
 * one-object stream on the tiled kernel (s3dg_set_stream_tiles). */
int s3dg_fill_controlled(s3dg_ctx *ctx, void *dst, uint64_t len, uint64_t dedup,
                         uint32_t f_num, uint32_t f_den, uint64_t entropy,
                         void *stream);
/* Blocks [blk_lo, blk_hi) of one `len`-byte object: block blk_lo lands at
 * dst.  Used to stream one large object through a smaller device buffer. */
int s3dg_fill_controlled_range(s3dg_ctx *ctx, void *dst, uint64_t len,
                               uint64_t blk_lo, uint64_t blk_hi, uint64_t dedup,
                               uint32_t f_num, uint32_t f_den, uint64_t entropy,
                               void *stream);
/* Seeded analogue of generate_random_data (src/data_gen.rs:102-132, whose
 * ThreadRng makes it unseedable): the context's base block tiled per 4 KiB
 * block, bytes [0, min(32, L)) then [L-32, L) when L > 2048 overwritten by
 * SmallRng::seed_from_u64(entropy + i).fill_bytes for block i. */
int s3dg_random_data(s3dg_ctx *ctx, void *dst, uint64_t len, uint64_t entropy, void *stream);
/* n equal-size objects, object j at dst + j*stride, entropy
 * s3dg_object_entropy(seed_base, first_obj + j). */
int s3dg_fill_controlled_stream(s3dg_ctx *ctx, void *dst, uint64_t obj_size,
                                uint64_t stride, uint64_t n_objs, uint64_t dedup,
                                uint32_t f_num, uint32_t f_den, uint64_t seed_base,
                                uint64_t first_obj, void *stream);
/* Mixed-size batch.  `descs` is a host array; it is consumed before return
 * (in sub-batches whose preparation overlaps the previous sub-batch's fill).
 * Descriptors are checked per sub-batch: when one is invalid the call fails
 * and the objects of earlier sub-batches may already be enqueued. */
int s3dg_fill_controlled_batch(s3dg_ctx *ctx, void *dst_base,
                               const s3dg_obj_desc *descs, uint64_t n, void *stream);
/* Keystream fill (generate_npz_bytes_raw x-fill, src/data_formats/npz.rs:376-383):
 * chunk k (chunk_bytes, last one ragged) of [dst, dst+len) =
 * Xoshiro256PlusPlus::seed_from_u64(seed_base + k).fill_bytes(chunk).
 * chunk_bytes: positive multiple of 128 (npz.rs uses 2 MiB). */
int s3dg_xoshiro_fill(s3dg_ctx *ctx, void *dst, uint64_t len, uint64_t chunk_bytes,
                      uint64_t seed_base, void *stream);
/* dgen-contract object ("DG1"): 1 MiB blocks [blk_lo, blk_hi) of
 * an obj_size-byte object, block blk_lo at dst.  Block i = Xoshiro256++ seeded
 * seed ^ ((i % U) * 0x9E3779B97F4A7C15) (U = s3dg_unique_blocks), its first
 * floor(L * f_num / f_den) bytes zero.  Behind DataGenerator/ObjectGen
 * (src/data_gen.rs:253-371) and dgen's generate_data; parity unpinned. */
int s3dg_dgen_fill(s3dg_ctx *ctx, void *dst, uint64_t obj_size, uint64_t blk_lo,
                   uint64_t blk_hi, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                   uint64_t seed, void *stream);
/* n_objs DG1 objects of obj_size bytes in one launch: object j at
 * dst + j*stride, seeded s3dg_object_entropy(seed_base, first_obj + j), i.e.
 * the bytes of n_objs s3dg_dgen_fill calls (ObjectGen / DataGenerator fanned
 * out over many objects).  stride >= obj_size, 16-byte aligned. */
int s3dg_dgen_fill_stream(s3dg_ctx *ctx, void *dst, uint64_t obj_size, uint64_t stride,
                          uint64_t n_objs, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                          uint64_t seed_base, uint64_t first_obj, void *stream);
/* Host helper: advance a Xoshiro256 state by n steps with the jump polynomial
 * the kernels use (test/diagnostic; no GPU needed). */
int s3dg_xoshiro_jump(uint64_t *state4, uint64_t n);
/* Write-only ceiling: fill `len` bytes with a constant using the same store
 * path (roofline denominator measured on the device). */
int s3dg_write_ceiling(s3dg_ctx *ctx, void *dst, uint64_t len, uint32_t pattern,
                       void *stream);
/* The same in the tiled fill shape (batch launch knobs, trailing loads of
 * the context's tile-map records, as k_fill_batch): the ceiling for tiled
 * batches and streams. */
int s3dg_write_ceiling_tiled(s3dg_ctx *ctx, void *dst, uint64_t len, uint32_t pattern, void *stream);
/* The store-only reference of the tiled fill itself: the launch
 * s3dg_fill_controlled_stream makes for len bytes of 8 MiB objects (same
 * tile records, grid, LDS image, barrier, stores and trailing record loads)
 * with the PRNG chain and the window patches compiled out.  Its bytes are
 * meaningless; it is the write ceiling the fill is measured against.
 * pace > 0 makes wave 0 of every workgroup idle pace x 128 cycles where the
 * fill plans its block (store issue paced like the fill's).
 * len < 8 MiB or a multiple of 8 MiB. */
int s3dg_write_ceiling_fill(s3dg_ctx *ctx, void *dst, uint64_t len, uint32_t pace, void *stream);

/* ---- memory / copy helpers ------------------------------------------------ */
int s3dg_device_alloc(s3dg_ctx *ctx, uint64_t bytes, void **out);
int s3dg_device_free(s3dg_ctx *ctx, void *p);
int s3dg_host_alloc_pinned(uint64_t bytes, void **out);
/* Pinned host memory placed on `device`'s NUMA node (allocated from a thread
 * bound to the GPU's local CPUs; falls back to default placement when sysfs
 * does not say).  Free with s3dg_host_free_pinned. */
int s3dg_host_alloc_pinned_local(int device, uint64_t bytes, void **out);
int s3dg_host_free_pinned(void *p);
/* Page-lock a caller's pageable buffer [buf, buf+len) (hipHostRegister, whole
 * 4 KiB pages) so that host-buffer calls inside it (s3dlio_fill_controlled_data
 * and the other host entry points; whole 4 KiB blocks, 16-byte aligned, up to
 * 16 MiB) are written by the kernel directly, as s3dg_host_alloc_pinned memory
 * (1 MiB: ~33 us against ~57 us through the bounce path).  Registrations that
 * overlap the range are dropped first; registering the same range again is a
 * no-op.  0 or a negative S3DG_E* status.
 * CONTRACT (hipHostRegister's): the buffer stays allocated until
 * s3dg_host_unregister.  Unmapped while registered, its GPU mapping goes with
 * its pages and the next call into it is a GPU memory fault.  The bindings
 * hold the buffer for the registration's lifetime (Python:
 * s3dlio_amd.register_host_buffer keeps an export of it; Rust:
 * HostRegistration<'a> borrows the slice).  Register a range
 * while no other thread's call is writing into it.
 * Replaces round 5's S3DLIO_HOST_REGISTER=1 sighting rule, which registered
 * buffers their owners did not know about. */
int s3dg_host_register(void *buf, uint64_t len);
/* Release the registration holding `buf` (NULL: every registration), after
 * calls still writing into it return.  Returns the number released (>= 0).
 * A call whose range overlaps a registration without lying inside it also
 * releases that registration (HIP cannot copy into a partly registered range). */
int s3dg_host_unregister(void *buf);
/* NUMA node of `device` from sysfs (-1 when unknown). */
int s3dg_device_numa_node(int device, int *node);
int s3dg_d2h_async(s3dg_ctx *ctx, void *host, const void *dev, uint64_t len, void *stream);
int s3dg_h2d_async(s3dg_ctx *ctx, void *dev, const void *host, uint64_t len, void *stream);
int s3dg_stream_create(s3dg_ctx *ctx, void **out);
int s3dg_stream_destroy(s3dg_ctx *ctx, void *stream);
/* Release the context's per-stream launch state (tile maps, batch staging) of
 * `stream`, after draining it: call before destroying a stream the context has
 * launched on, so short-lived streams do not accumulate device memory.
 * s3dg_stream_destroy does this itself.  No-op for an unknown stream.  A
 * launch on `stream` from another thread may race with the release: it
 * completes, and the last holder of the state drains the stream and frees it.
 * s3dg_stream_destroy must not run while another thread still uses `stream`
 * (the HIP stream itself is destroyed, even when the drain reports an error). */
int s3dg_stream_release(s3dg_ctx *ctx, void *stream);
int s3dg_stream_state_count(s3dg_ctx *ctx, uint64_t *n);
int s3dg_sync(s3dg_ctx *ctx, void *stream);   /* stream NULL: whole device */
int s3dg_device_count(int *out);

/* ---- CRC-32 and NPZ (src/data_formats/npz.rs:322-434) --------------------- */
/* CRC-32 (IEEE, crc32fast / zlib.crc32) of dev[0, len); synchronous on `stream`. */
int s3dg_crc32(s3dg_ctx *ctx, const void *dev, uint64_t len, void *stream, uint32_t *out);
/* zlib crc32_combine: CRC of A||B from crc(A), crc(B), |B| (host). */
uint32_t s3dg_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
/* Host CRC-32 update (crc32fast::Hasher semantics: start from 0). */
uint32_t s3dg_crc32_host(uint32_t crc, const uint8_t *p, uint64_t n);
/* Byte size of generate_npz_bytes_raw(shape, dtype, num_samples). */
int s3dg_npz_size(const uint64_t *shape, int ndim, const char *dtype, uint64_t num_samples,
                  uint64_t *total);
/* generate_npz_bytes_raw into a host buffer of >= s3dg_npz_size bytes:
 * byte-identical archive (x.npy keystream + CRC on the GPU, framing on host). */
int s3dg_npz_build(s3dg_ctx *ctx, const uint64_t *shape, int ndim, const char *dtype,
                   uint64_t num_samples, uint8_t *out, uint64_t out_len);

/* ---- streaming generator (DataGenerator / ObjectGen / PyO3 Generator) ----- */
/* One object of `size` bytes in the DG1 layout, generated on a host slot's
 * GPU (taken round-robin at creation) and streamed into host buffers.  has_seed=0: time + counter
 * entropy like DataGenerator::new(None) (src/data_gen.rs:271-291).
 * compress/dedup 0 are treated as 1 (src/data_gen_alt.rs:108-109). */
typedef struct s3dg_gen s3dg_gen;
int s3dg_gen_create(uint64_t size, uint64_t dedup, uint64_t compress, int has_seed,
                    uint64_t seed, s3dg_gen **out);
int s3dg_gen_create_ratio(uint64_t size, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                          int has_seed, uint64_t seed, s3dg_gen **out);
int s3dg_gen_destroy(s3dg_gen *gen);
/* ObjectGenAlt::fill_chunk (src/data_gen_alt.rs:122): next min(cap, remaining)
 * bytes into buf; *written = 0 once complete. */
int s3dg_gen_fill_chunk(s3dg_gen *gen, uint8_t *buf, uint64_t cap, uint64_t *written);
/* Random access: bytes [pos, pos+n) of the object (does not move position). */
int s3dg_gen_fill_at(s3dg_gen *gen, uint8_t *buf, uint64_t pos, uint64_t n);
int s3dg_gen_is_complete(s3dg_gen *gen);
uint64_t s3dg_gen_position(s3dg_gen *gen);
uint64_t s3dg_gen_total_size(s3dg_gen *gen);
uint64_t s3dg_gen_seed(s3dg_gen *gen);
/* The host slot the generator runs on (s3dg_host_slot_device gives its GPU). */
int s3dg_gen_slot(s3dg_gen *gen);
int s3dg_gen_reset(s3dg_gen *gen);
/* generate_data / generate_controlled_data_alt one-shot into buf. */
int s3dg_generate_data(uint8_t *buf, uint64_t size, uint64_t dedup, uint64_t compress,
                       int has_seed, uint64_t seed);

/* ---- object assembly: generate_object (src/data_gen.rs:29-94) ------------ */
enum { S3DG_OBJ_NPZ = 0, S3DG_OBJ_TFRECORD = 1, S3DG_OBJ_HDF5 = 2, S3DG_OBJ_RAW = 3 };
enum { S3DG_MODE_STREAMING = 0, S3DG_MODE_SINGLE_PASS = 1 };
/* Bytes generate_object produces for (type, elements, element_size). */
int s3dg_object_size(int type, uint64_t elements, uint64_t element_size, uint64_t *out);
/* generate_object(&Config) into `out` (>= s3dg_object_size bytes):
 * use_controlled=0 -> generate_random_data payload, else the dgen-contract
 * payload; then build_raw / build_tfrecord / build_npz.  HDF5 -> S3DG_EINVAL
 * (as a reference build without the hdf5 feature).  has_seed=0 reproduces
 * the reference's non-deterministic entropy. */
int s3dg_generate_object(int type, uint64_t elements, uint64_t element_size, int use_controlled,
                         uint64_t dedup, uint64_t compress, int mode, int has_seed, uint64_t seed,
                         uint8_t *out, uint64_t out_len, uint64_t *written);
/* build_tfrecord_with_index (src/data_formats/tfrecord.rs:47-75): records of
 * record_size bytes from `data` -> out (records * (16 + record_size) bytes;
 * may alias data shifted by 12 for one record); index_out (nullable) gets
 * 16 bytes <offset u64, length u64> per record. */
int s3dg_build_tfrecord(uint64_t records, uint64_t record_size, const uint8_t *data, uint8_t *out,
                        uint8_t *index_out);
/* build_npz (src/data_formats/npz.rs:114-132): "data.npy" in a stored ZIP. */
int s3dg_npz_legacy_size(uint64_t elements, uint64_t data_len, uint64_t *out);
int s3dg_build_npz(uint64_t elements, const uint8_t *data, uint64_t data_len, uint8_t *out,
                   uint64_t out_len);

/* ---- put pipeline: per-object payloads -> files -------- */
/* Replaces put_objects_with_random_data_and_type (src/s3_utils.rs:1717-1750)
 * + put_objects_parallel_with_progress (:1812-1868) + FileSystemObjectStore::put
 * (src/file_store.rs:550-569) for file:// targets, with one payload PER OBJECT
 * (the reference PUTs one buffer to every URI).  Object j (paths[j], a plain
 * file-system path: the file:// prefix already stripped) is framed as
 * object_type with elements = 1, element_size = size (python_core_api.rs:804),
 * its payload generated on the GPU with entropy object_entropy(seed_base, j):
 *   S3DG_PAYLOAD_CONTROLLED  fill_controlled_data layout (data_gen.rs:151-224)
 *   S3DG_PAYLOAD_RANDOM      generate_random_data layout (data_gen.rs:102-132)
 *   S3DG_PAYLOAD_DGEN        the DG1 dgen-contract stream
 * Parent directories are created; files are truncated.  max_in_flight writer
 * threads (0 -> 64) write from a pinned host ring while the GPU generates the
 * next chunk.  crc_out (nullable, n entries) receives the CRC-32 (crc32fast)
 * of each whole file as written (StreamingDataWriter::checksum,
 * src/streaming_writer.rs:183-186).  File-system errors -> S3DG_EIO. */
enum { S3DG_PAYLOAD_CONTROLLED = 0, S3DG_PAYLOAD_RANDOM = 1, S3DG_PAYLOAD_DGEN = 2 };
typedef struct {
    uint64_t objects;       /* files written */
    uint64_t bytes;         /* bytes written (payload + framing) */
    double seconds;         /* wall time of the call */
    double gpu_seconds;     /* time the generator thread waited on the GPU (gen + CRC + D2H) */
} s3dg_put_stats;
int s3dg_put_objects(s3dg_ctx *ctx, const char *const *paths, uint64_t n, uint64_t size,
                     int object_type, int payload, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                     uint64_t seed_base, uint32_t max_in_flight, uint32_t *crc_out,
                     s3dg_put_stats *stats);
/* Same over several contexts (GPUs): object j is generated by context
 * j * nctx / n's lane (contiguous ranges), each lane with its own device
 * chunks, streams and pinned ring on its GPU's NUMA node, one shared writer
 * pool.  Files and checksums are identical for any nctx; two contexts on one
 * device run two lanes on it. */
int s3dg_put_objects_multi(s3dg_ctx *const *ctxs, uint32_t nctx, const char *const *paths,
                           uint64_t n, uint64_t size, int object_type, int payload, uint64_t dedup,
                           uint32_t f_num, uint32_t f_den, uint64_t seed_base, uint32_t max_in_flight,
                           uint32_t *crc_out, s3dg_put_stats *stats);

/* ---- host-buffer drop-ins (src/data_gen.rs:151 signature) ---------------- */
/* The host-buffer entry points (s3dlio_*, s3dg_gen_*, s3dg_generate_data,
 * s3dg_generate_object) run on a pool of SLOTS: one per GPU by default, each
 * with its own context, base-block copies and staging sets.  Every call takes
 * a slot round-robin (a generator keeps its slot); calls on different slots
 * run on different GPUs concurrently, and a call of >= 256 MiB is cut into
 * one range per slot generated in parallel.  Bytes never depend on the slot.
 * Slot devices: env S3DLIO_GPU_DEVICE=k pins every call to GPU k;
 * S3DLIO_GPU_DEVICES=a,b,... lists them (repeats: several slots on one GPU);
 * neither: every visible GPU, or, in one rank of a multi-process job
 * (WORLD_SIZE > 1 and LOCAL_RANK set), that rank's GPU (LOCAL_RANK mod the
 * device count) only.  Env S3DLIO_HOST_D2H=staged copies through pinned
 * bounce buffers instead of straight into the caller's memory. */
/* The slot device list for the given env values and device count (pure
 * function; no GPU needed).  *n <= cap entries written to out. */
int s3dg_host_parse_devices(const char *pin, const char *list, int ndev, int *out, int cap, int *n);
/* The same with the multi-process job's LOCAL_RANK / WORLD_SIZE values (NULL:
 * unset); the library's own slot list is this function of its environment. */
int s3dg_host_parse_devices_env(const char *pin, const char *list, const char *local_rank,
                                const char *world_size, int ndev, int *out, int cap, int *n);
int s3dg_host_slot_count(int *out);
int s3dg_host_slot_device(int slot, int *device);
/* The slot's context (owned by the pool: never destroy it); slot < 0 takes
 * the next slot round-robin. */
int s3dg_host_slot_context(int slot, s3dg_ctx **out);
/* generate_random_data(size) (src/data_gen.rs:102): seeded analogue layout
 * with time entropy and a per-process random BASE_BLOCK. */
int s3dlio_generate_random_data(uint8_t *buf, size_t size);
/* fill_controlled_data(buf, dedup, compress): time-based entropy and a
 * per-process random base block, exactly as the reference; generated on the
 * host slots' GPUs (above) and copied into `buf`.  Empty buffer: no-op. */
int s3dlio_fill_controlled_data(uint8_t *buf, size_t len, size_t dedup, size_t compress);
/* Seeded sibling: entropy replaces call_entropy; base4096 (nullable)
 * replaces A_BASE_BLOCK (NULL = a context's default base block, seed
 * 0xBA5EB10C00000000). */
int s3dlio_fill_controlled_data_seeded(uint8_t *buf, size_t len, size_t dedup,
                                       size_t compress, uint64_t entropy,
                                       const uint8_t *base4096);

const char *s3dg_last_error(void);
const char *s3dg_version(void);
/* The 16-hex-digit digest of the sources the library was built from
 * (s3dlio_amd/build.py source_digest); bench.py stamps it and refuses a
 * library whose digest differs from the tree it runs in. */
const char *s3dg_build_digest(void);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* S3DLIO_GPU_H */
