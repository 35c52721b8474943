// s3dg_capi.cpp — C ABI (include/s3dlio_gpu.h) over the gfx950 kernels.
//
// Host-side parameter math follows /root/reference/src/data_gen.rs:151-224:
// unique_blocks (:162-167), (f_num, f_den) (:169-173), floor_len/rem
// (:174-175).  No CPU generation path exists in this library: every byte is
// produced by a HIP kernel, and a missing/failed GPU is an error.
#include "s3dg_internal.h"
#include "s3dg_jump.h"

namespace s3dg {
uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
uint32_t crc32_host_update(uint32_t crc, const uint8_t *p, uint64_t n);
hipError_t crc32_device(const uint8_t *dev, uint64_t len, hipStream_t s, uint32_t *out,
                        void **tab_cache, uint32_t **seg_cache, uint64_t *seg_cap);
}  // namespace s3dg
#include "s3dlio_gpu.h"

#include <sys/random.h>
#include <time.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace s3dg;

constexpr int kDefaultOccStream = 14, kDefaultOccBatch = 0;
constexpr uint32_t kDefaultPrefetch = 256;   // in 64-block units; > resident workgroups / 64
constexpr int kDefaultStreamTiles = 1;
constexpr uint64_t kStreamTilesMinBlocks = 16384;   // smaller streams: 2D kernel, no tile-map launch
constexpr int kDefaultStoreStream = kStoreNTSC1, kDefaultStoreBatch = kStoreSC1;
constexpr uint64_t kDefaultKsMinDraws[2] = {2048, 1024};   // npz keystream, DG1
constexpr uint64_t kKsMinSpan = 256;          // fewest draws per lane for small launches
// measured on MI355X (tools/k2_lab.py): 512-B row pieces and sc1 stores for
// the plain keystream; 128-B pieces, 2-wave workgroups, 1024 draws per lane
// and plain stores for DG1 (zero-prefixed 1 MiB blocks: with 128 lanes per
// block, whole waves fall inside the prefix and skip the PRNG)
constexpr KsShape kDefaultKsShape[2] = {{64, 4, 0, kStoreSC1}, {16, 2, 0, kStorePlain}};

struct s3dg_ctx {
    int device = 0;
    int cus = 256;                     // compute units (sizes small keystream launches)
    // store cache policy: sc1 (write, then drop the line from
    // L2) for batches, nt sc1 for streams, measured best
    int store_stream = kDefaultStoreStream, store_batch = kDefaultStoreBatch;
    int waves_per_block = 0;           // 0 = auto: 2 for streams, 1 for batches (measured)
    // resident fill workgroups per CU (0 = hardware max); measured on MI355X
    // (DESIGN.md §5.1): 14 for 2-wave stream blocks, no cap for 1-wave batch blocks
    int occ_stream = kDefaultOccStream, occ_batch = kDefaultOccBatch;
    uint32_t prefetch_tiles = kDefaultPrefetch;   // batch tile-record prefetch distance
    uint32_t tile_shift = 0;           // batch tile = 2^tile_shift blocks; 0 = per launch
    // k_keystream launch shapes, [0] npz keystream, [1] DG1
    KsShape ks[2] = {kDefaultKsShape[0], kDefaultKsShape[1]};
    uint64_t ks_min_draws[2] = {kDefaultKsMinDraws[0], kDefaultKsMinDraws[1]};   // draws per lane
    void *base_dev = nullptr;          // 4 KiB base block in HBM
    uint8_t base_host[kBlk];
    // batch descriptor table (device) + pinned staging, grown on demand
    ObjEntry *tab_dev = nullptr;
    ObjEntry *tab_host = nullptr;
    uint64_t tab_cap = 0;
    TileRec *tile_obj = nullptr;       // per-tile records (device)
    uint64_t tile_cap = 0;
    hipEvent_t tab_free = nullptr;     // staging may be rewritten once this fires
    hipEvent_t tile_free = nullptr;    // tile map may be rewritten once this fires
    int stream_tiles = kDefaultStreamTiles;   // uniform streams through the tiled batch kernel
    std::map<uint64_t, uint64_t *> jtabs;   // (lpc << 32 | span) -> device jump table
    void *crc_tab = nullptr;           // slicing-by-8 tables (device)
    uint32_t *crc_seg = nullptr;       // per-segment CRCs (device)
    uint64_t crc_seg_cap = 0;
    std::mutex crc_mu;
    std::mutex mu;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hipfail(hipError_t e, const char *what) {
    return fail(S3DG_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return hipfail(e_, what); \
    } while (0)

// SmallRng seeding + Xoshiro256++ on the host, only to derive a base block
// from a seed (4 KiB, once per set call).
uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
void base_from_seed(uint64_t seed, uint8_t *out) {
    uint64_t x = seed, s[4];
    for (int k = 0; k < 4; ++k) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        s[k] = z ^ (z >> 31);
    }
    for (uint32_t off = 0; off < kBlk; off += 8) {
        const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t;
        s[3] = rotl(s[3], 45);
        std::memcpy(out + off, &r, 8);   // little-endian host
    }
}

constexpr uint64_t kDefaultBaseSeed = 0xBA5EB10C00000000ull;

// Entry points: a null context is an error; the context's device is made
// current for the call and the caller's current device restored afterwards.
#define CTX_SCOPE(c)                                                   \
    if (!(c)) return fail(S3DG_EINVAL, "null context");                \
    DeviceScope dscope_((c)->device);                                  \
    if (!dscope_.ok()) return hipfail(dscope_.err, "hipSetDevice")

int make_prefix(uint64_t nblocks, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                PrefixParams *pp) {
    if (f_den == 0) return fail(S3DG_EINVAL, "f_den must be >= 1");
    if (f_num >= f_den) return fail(S3DG_EINVAL, "f_num must be < f_den (zero ratio < 1)");
    if (nblocks > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "object larger than 2^32 blocks");
    const uint64_t tot = (uint64_t)f_num * kBlk;
    const uint64_t U = s3dg_unique_blocks(nblocks, dedup);
    pp->unique = U == nblocks ? 0xFFFFFFFFu : (uint32_t)U;
    pp->floor_len = (uint32_t)(tot / f_den);
    pp->rem = (uint32_t)(tot % f_den);
    pp->f_den = f_den;
    pp->m_unique = fastmod_magic(pp->unique == 0xFFFFFFFFu ? 1u : pp->unique);
    pp->m_fden = fastmod_magic(f_den);
    return S3DG_OK;
}

LaunchCfg cfg_for(s3dg_ctx *c, bool batch = false) {
    LaunchCfg lc;
    lc.store = batch ? c->store_batch : c->store_stream;
    lc.waves_per_block = c->waves_per_block ? c->waves_per_block : (batch ? 1 : 2);
    lc.dyn_lds = occupancy_lds(batch ? c->occ_batch : c->occ_stream, kFillStaticLds);
    lc.prefetch_tiles = batch ? c->prefetch_tiles : 0;
    return lc;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// Batch tile size: every object's last tile is ragged, and its blocks past
// the object's end are workgroups that start, load the record and exit.
// Smaller tiles cut those, at one 64-B record (and one more record miss per
// XCD) per tile.  Pick the tile size that minimises launched workgroups +
// kTileCost x records.
constexpr uint64_t kTileCost = 2;

uint32_t pick_tile_shift(const uint64_t (&ntiles)[kTileShiftMax + 1]) {
    uint32_t best = kTileShiftMax;
    uint64_t best_cost = UINT64_MAX;
    for (uint32_t sh = kTileShiftMax; sh >= kTileShiftMin; --sh) {
        const uint64_t cost = (ntiles[sh] << sh) + kTileCost * ntiles[sh];
        if (cost < best_cost) { best_cost = cost; best = sh; }
    }
    return best;
}

}  // namespace

extern "C" {

const char *s3dg_last_error(void) { return g_err.c_str(); }
const char *s3dg_version(void) { return "s3dlio_amd 0.1.0 (gfx950)"; }

uint64_t s3dg_unique_blocks(uint64_t nblocks, uint64_t dedup) {
    const uint64_t d = dedup == 0 ? 1 : dedup;
    if (d <= 1) return nblocks;
    double r = std::round((double)nblocks / (double)d);   // f64::round, half away
    if (r < 1.0) r = 1.0;
    return (uint64_t)r;
}

int s3dg_compress_ratio(uint64_t compress, uint32_t *f_num, uint32_t *f_den) {
    if (!f_num || !f_den) return fail(S3DG_EINVAL, "null output");
    if (compress > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "compress must fit in 32 bits");
    if (compress > 1) { *f_num = (uint32_t)(compress - 1); *f_den = (uint32_t)compress; }
    else { *f_num = 0; *f_den = 1; }
    return S3DG_OK;
}

uint64_t s3dg_object_entropy(uint64_t seed_base, uint64_t j) { return seed_base + (j << 32); }

int s3dg_device_count(int *out) {
    if (!out) return fail(S3DG_EINVAL, "null output");
    HIP_TRY(hipGetDeviceCount(out), "hipGetDeviceCount");
    return S3DG_OK;
}

int s3dg_ctx_create(int device, s3dg_ctx **out) {
    if (!out) return fail(S3DG_EINVAL, "null output");
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n), "hipGetDeviceCount");
    if (device < 0 || device >= n) return fail(S3DG_EINVAL, "device index out of range");
    DeviceScope ds(device);
    if (!ds.ok()) return hipfail(ds.err, "hipSetDevice");
    s3dg_ctx *c = new s3dg_ctx();
    c->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->cus = cus;
    hipError_t e = hipMalloc(&c->base_dev, kBlk);
    if (e != hipSuccess) { delete c; return hipfail(e, "hipMalloc(base block)"); }
    e = hipEventCreateWithFlags(&c->tab_free, hipEventDisableTiming);
    if (e != hipSuccess) { (void)hipFree(c->base_dev); delete c; return hipfail(e, "hipEventCreate"); }
    e = hipEventCreateWithFlags(&c->tile_free, hipEventDisableTiming);
    if (e != hipSuccess) { s3dg_ctx_destroy(c); return hipfail(e, "hipEventCreate"); }
    base_from_seed(kDefaultBaseSeed, c->base_host);
    e = hipMemcpy(c->base_dev, c->base_host, kBlk, hipMemcpyHostToDevice);
    if (e != hipSuccess) { s3dg_ctx_destroy(c); return hipfail(e, "hipMemcpy(base block)"); }
    *out = c;
    return S3DG_OK;
}

int s3dg_ctx_destroy(s3dg_ctx *c) {
    if (!c) return S3DG_OK;
    DeviceScope ds(c->device);
    (void)hipDeviceSynchronize();
    if (c->base_dev) (void)hipFree(c->base_dev);
    if (c->tab_dev) (void)hipFree(c->tab_dev);
    if (c->tab_host) (void)hipHostFree(c->tab_host);
    if (c->tile_obj) (void)hipFree(c->tile_obj);
    for (auto &kv : c->jtabs) (void)hipFree(kv.second);
    if (c->crc_tab) (void)hipFree(c->crc_tab);
    if (c->crc_seg) (void)hipFree(c->crc_seg);
    if (c->tab_free) (void)hipEventDestroy(c->tab_free);
    if (c->tile_free) (void)hipEventDestroy(c->tile_free);
    delete c;
    return S3DG_OK;
}

int s3dg_set_base_block(s3dg_ctx *c, const uint8_t *base) {
    CTX_SCOPE(c);
    if (!base) return fail(S3DG_EINVAL, "null base block");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");   // no launch may read the old block
    std::memcpy(c->base_host, base, kBlk);
    HIP_TRY(hipMemcpy(c->base_dev, c->base_host, kBlk, hipMemcpyHostToDevice), "hipMemcpy(base)");
    return S3DG_OK;
}

int s3dg_set_base_block_seed(s3dg_ctx *c, uint64_t seed) {
    uint8_t b[kBlk];
    base_from_seed(seed, b);
    return s3dg_set_base_block(c, b);
}

int s3dg_get_base_block(s3dg_ctx *c, uint8_t *out) {
    if (!c || !out) return fail(S3DG_EINVAL, "null argument");
    std::memcpy(out, c->base_host, kBlk);
    return S3DG_OK;
}

int s3dg_set_waves_per_block(s3dg_ctx *c, int waves) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (waves != 0 && waves != 1 && waves != 2 && waves != 4) return fail(S3DG_EINVAL, "waves per block must be 1, 2 or 4");
    c->waves_per_block = waves;
    return S3DG_OK;
}

int s3dg_set_nontemporal(s3dg_ctx *c, int on) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    c->store_stream = on ? kStoreNT : kDefaultStoreStream;
    c->store_batch = on ? kStoreNT : kDefaultStoreBatch;
    return S3DG_OK;
}

int s3dg_set_store_policy(s3dg_ctx *c, int stream_policy, int batch_policy) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (stream_policy > kStoreNTSC1 || batch_policy > kStoreNTSC1)
        return fail(S3DG_EINVAL, "store policy must be 0 (plain), 1 (nt), 2 (sc1), 3 (nt sc1) or negative (default)");
    c->store_stream = stream_policy < 0 ? kDefaultStoreStream : stream_policy;
    c->store_batch = batch_policy < 0 ? kDefaultStoreBatch : batch_policy;
    return S3DG_OK;
}

int s3dg_set_occupancy(s3dg_ctx *c, int stream_wgs_per_cu, int batch_wgs_per_cu) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (stream_wgs_per_cu > 40 || batch_wgs_per_cu > 40)
        return fail(S3DG_EINVAL, "workgroups per CU must be at most 40");
    c->occ_stream = stream_wgs_per_cu < 0 ? kDefaultOccStream : stream_wgs_per_cu;
    c->occ_batch = batch_wgs_per_cu < 0 ? kDefaultOccBatch : batch_wgs_per_cu;
    return S3DG_OK;
}

int s3dg_set_batch_prefetch(s3dg_ctx *c, uint32_t tiles) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    c->prefetch_tiles = tiles == UINT32_MAX ? kDefaultPrefetch : tiles;
    return S3DG_OK;
}

int s3dg_set_batch_tile(s3dg_ctx *c, uint32_t blocks) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    uint32_t sh = 0;
    if (blocks != 0) {
        while ((1u << sh) < blocks) ++sh;
        if ((1u << sh) != blocks || sh < kTileShiftMin || sh > kTileShiftMax)
            return fail(S3DG_EINVAL, "tile blocks must be 0 (per launch), 8, 16, 32 or 64");
    }
    c->tile_shift = sh;
    return S3DG_OK;
}

int s3dg_set_keystream_shape(s3dg_ctx *c, int mode, int draws, int waves, int wgs_per_cu,
                             uint64_t min_lane_draws, int store_policy) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (mode != 0 && mode != 1) return fail(S3DG_EINVAL, "mode must be 0 (keystream) or 1 (dgen)");
    if (draws != 0 && draws != 16 && draws != 32 && draws != 64)
        return fail(S3DG_EINVAL, "draws per stage must be 16, 32 or 64");
    if (waves != 0 && waves != 1 && waves != 2 && waves != 4) return fail(S3DG_EINVAL, "waves must be 1, 2 or 4");
    if (wgs_per_cu < 0 || wgs_per_cu > 40) return fail(S3DG_EINVAL, "workgroups per CU must be 0..40");
    if (min_lane_draws != 0 && min_lane_draws < 64) return fail(S3DG_EINVAL, "min_lane_draws must be >= 64");
    if (store_policy > kStoreNTSC1) return fail(S3DG_EINVAL, "store policy must be 0, 1, 2, 3 or negative");
    std::lock_guard<std::mutex> g(c->mu);
    const KsShape &def = kDefaultKsShape[mode];
    c->ks[mode].draws = draws ? draws : def.draws;
    c->ks[mode].waves = waves ? waves : def.waves;
    c->ks[mode].wgs_per_cu = wgs_per_cu;
    c->ks[mode].store = store_policy < 0 ? def.store : store_policy;
    c->ks_min_draws[mode] = min_lane_draws ? min_lane_draws : kDefaultKsMinDraws[mode];
    return S3DG_OK;
}

int s3dg_query_keystream_occupancy(s3dg_ctx *c, int mode, int *wgs_per_cu) {
    CTX_SCOPE(c);
    if (!wgs_per_cu || (mode != 0 && mode != 1)) return fail(S3DG_EINVAL, "bad argument");
    HIP_TRY(keystream_occupancy(c->ks[mode], wgs_per_cu), "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    return S3DG_OK;
}

int s3dg_query_occupancy(s3dg_ctx *c, int batch, int *wgs_per_cu) {
    CTX_SCOPE(c);
    if (!wgs_per_cu) return fail(S3DG_EINVAL, "null output");
    HIP_TRY(fill_occupancy(cfg_for(c, batch != 0), batch != 0, wgs_per_cu), "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    return S3DG_OK;
}

// The tile map (c->tile_obj) is shared by the context's batch and tiled
// stream launches, which may be on different streams: grow it only once the
// last launch reading it is done, and order the next k_tile_map after that
// launch on the device (tile_free is recorded after every reader).  Caller
// holds c->mu until it has recorded tile_free.
static int tile_map_acquire(s3dg_ctx *c, uint64_t tiles, hipStream_t s) {
    if (tiles > c->tile_cap) {
        HIP_TRY(hipEventSynchronize(c->tile_free), "hipEventSynchronize(tile map)");
        if (c->tile_obj) (void)hipFree(c->tile_obj);
        c->tile_obj = nullptr; c->tile_cap = 0;
        const uint64_t cap = tiles < 4096 ? 4096 : tiles + tiles / 4;
        HIP_TRY(hipMalloc(&c->tile_obj, cap * sizeof(TileRec)), "hipMalloc(tile map)");
        c->tile_cap = cap;
    }
    HIP_TRY(hipStreamWaitEvent(s, c->tile_free, 0), "hipStreamWaitEvent(tile map)");
    return S3DG_OK;
}

// n_objs objects of obj_size bytes at dst + j*stride, entropy seed_base +
// ((first_obj + j) << 32), prefix parameters pp.  Large streams whose objects
// all start on the same 4 KiB granule (mod 8) run through the tiled batch
// kernel; the rest through the 2D stream kernel.
static int fill_uniform(s3dg_ctx *c, uint8_t *dst, uint64_t obj_size, uint64_t stride, uint64_t n_objs,
                        const PrefixParams &pp, uint64_t seed_base, uint64_t first_obj, hipStream_t s) {
    const uint64_t nb = (obj_size + kBlk - 1) / kBlk;
    const uint32_t lead = (uint32_t)(((uintptr_t)dst >> 12) & 7);
    if (c->stream_tiles && (n_objs == 1 || stride % (8 * kBlk) == 0) && n_objs * nb >= kStreamTilesMinBlocks &&
        nb + lead < (1ull << 31)) {
        uint64_t ntiles[kTileShiftMax + 1] = {};
        for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh)
            ntiles[sh] = n_objs * ((nb + lead + (1ull << sh) - 1) >> sh);
        const uint32_t tshift = c->tile_shift ? c->tile_shift : pick_tile_shift(ntiles);
        const uint64_t tpo = (nb + lead + (1ull << tshift) - 1) >> tshift;
        std::lock_guard<std::mutex> g(c->mu);
        if (int r = tile_map_acquire(c, n_objs * tpo, s)) return r;
        HIP_TRY(launch_fill_uniform_tiles(cfg_for(c, true), dst, obj_size, stride, n_objs, (uint32_t)tpo, tshift,
                                          lead, seed_base + (first_obj << 32), pp, c->tile_obj, c->base_dev, s),
                "launch k_fill_batch(stream)");
        HIP_TRY(hipEventRecord(c->tile_free, s), "hipEventRecord");
        return S3DG_OK;
    }
    HIP_TRY(launch_fill_stream(cfg_for(c), dst, obj_size, stride, n_objs, 0, (uint32_t)nb, seed_base, first_obj,
                               pp, c->base_dev, s),
            "launch k_fill_stream");
    return S3DG_OK;
}

int s3dg_fill_controlled_range(s3dg_ctx *c, void *dst, uint64_t len, uint64_t blk_lo,
                               uint64_t blk_hi, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                               uint64_t entropy, void *stream) {
    CTX_SCOPE(c);
    if (len == 0) return S3DG_OK;                                   // :154-156
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    if (blk_hi > nb) blk_hi = nb;
    if (blk_lo >= blk_hi) return S3DG_OK;
    if (!dst || !aligned16(dst)) return fail(S3DG_EINVAL, "dst must be a 16-byte aligned device pointer");
    // a whole large buffer is a one-object stream: the tiled kernel (entropy
    // of stream object 0 with seed_base = entropy is entropy itself)
    if (blk_lo == 0 && blk_hi == nb && c->stream_tiles && nb >= kStreamTilesMinBlocks)
        return s3dg_fill_controlled_stream(c, dst, len, (len + 15) & ~15ull, 1, dedup, f_num, f_den, entropy, 0,
                                           stream);
    PrefixParams pp;
    if (int r = make_prefix(nb, dedup, f_num, f_den, &pp)) return r;
    HIP_TRY(launch_fill_stream(cfg_for(c), (uint8_t *)dst, len, 0, 1, (uint32_t)blk_lo,
                               (uint32_t)blk_hi, entropy, 0, pp, c->base_dev,
                               (hipStream_t)stream),
            "launch k_fill_stream");
    return S3DG_OK;
}

int s3dg_random_data(s3dg_ctx *c, void *dst, uint64_t len, uint64_t entropy, void *stream) {
    CTX_SCOPE(c);
    if (len == 0) return S3DG_OK;
    if (!dst || !aligned16(dst)) return fail(S3DG_EINVAL, "dst must be a 16-byte aligned device pointer");
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    if (nb > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "object larger than 2^32 blocks");
    PrefixParams pp{};
    pp.unique = 0xFFFFFFFFu;            // block i seeded entropy + i
    pp.f_den = 0;                       // random-data layout
    pp.m_unique = fastmod_magic(1);
    pp.m_fden = fastmod_magic(1);
    return fill_uniform(c, (uint8_t *)dst, len, (len + 15) & ~15ull, 1, pp, entropy, 0, (hipStream_t)stream);
}

// The context's device (callers make it current with a DeviceScope).
int s3dg_internal_ctx_device(s3dg_ctx *c, int *dev) {
    if (!c || !dev) return fail(S3DG_EINVAL, "null context");
    *dev = c->device;
    return S3DG_OK;
}

// Chunk of n_objs equal objects for the put pipeline: blocks [blk_lo, blk_hi)
// of objects first_obj..first_obj+n_objs-1, object k's block blk_lo at
// dst + k*stride; controlled layout or (random_layout) generate_random_data's.
int s3dg_internal_fill_chunk(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride,
                             uint64_t n_objs, uint64_t blk_lo, uint64_t blk_hi, int random_layout,
                             uint64_t dedup, uint32_t f_num, uint32_t f_den, uint64_t seed_base,
                             uint64_t first_obj, void *stream) {
    CTX_SCOPE(c);
    if (obj_size == 0 || n_objs == 0) return S3DG_OK;
    const uint64_t nb = (obj_size + kBlk - 1) / kBlk;
    if (blk_hi > nb) blk_hi = nb;
    if (blk_lo >= blk_hi) return S3DG_OK;
    if (!dst || !aligned16(dst) || (stride & 15u)) return fail(S3DG_EINVAL, "dst and stride must be 16-byte aligned");
    PrefixParams pp{};
    if (random_layout) {
        if (nb > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "object larger than 2^32 blocks");
        pp.unique = 0xFFFFFFFFu;
        pp.f_den = 0;
        pp.m_unique = fastmod_magic(1);
        pp.m_fden = fastmod_magic(1);
    } else if (int r = make_prefix(nb, dedup, f_num, f_den, &pp)) {
        return r;
    }
    HIP_TRY(launch_fill_stream(cfg_for(c), (uint8_t *)dst, obj_size, stride, n_objs, (uint32_t)blk_lo,
                               (uint32_t)blk_hi, seed_base, first_obj, pp, c->base_dev, (hipStream_t)stream),
            "launch k_fill_stream(put chunk)");
    return S3DG_OK;
}

int s3dg_fill_controlled(s3dg_ctx *c, void *dst, uint64_t len, uint64_t dedup, uint32_t f_num,
                         uint32_t f_den, uint64_t entropy, void *stream) {
    return s3dg_fill_controlled_range(c, dst, len, 0, ~0ull, dedup, f_num, f_den, entropy, stream);
}

int s3dg_fill_controlled_stream(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride,
                                uint64_t n_objs, uint64_t dedup, uint32_t f_num, uint32_t f_den,
                                uint64_t seed_base, uint64_t first_obj, void *stream) {
    CTX_SCOPE(c);
    if (obj_size == 0 || n_objs == 0) return S3DG_OK;
    if (!dst || !aligned16(dst) || (stride & 15u))
        return fail(S3DG_EINVAL, "dst and stride must be 16-byte aligned");
    if (n_objs > 1 && stride < obj_size) return fail(S3DG_EINVAL, "stride < obj_size: objects overlap");
    const uint64_t nb = (obj_size + kBlk - 1) / kBlk;
    PrefixParams pp;
    if (int r = make_prefix(nb, dedup, f_num, f_den, &pp)) return r;
    return fill_uniform(c, (uint8_t *)dst, obj_size, stride, n_objs, pp, seed_base, first_obj, (hipStream_t)stream);
}

int s3dg_set_stream_tiles(s3dg_ctx *c, int on) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    c->stream_tiles = on < 0 ? kDefaultStreamTiles : (on != 0);
    return S3DG_OK;
}

int s3dg_fill_controlled_batch(s3dg_ctx *c, void *dst_base, const s3dg_obj_desc *d, uint64_t n,
                               void *stream) {
    CTX_SCOPE(c);
    if (n == 0) return S3DG_OK;
    if (!d) return fail(S3DG_EINVAL, "null descriptor array");
    if (!dst_base || !aligned16(dst_base)) return fail(S3DG_EINVAL, "dst_base must be 16-byte aligned");
    std::lock_guard<std::mutex> g(c->mu);
    // the previous batch's upload must have left the pinned staging table
    HIP_TRY(hipEventSynchronize(c->tab_free), "hipEventSynchronize");
    if (n > c->tab_cap) {
        if (c->tab_dev) (void)hipFree(c->tab_dev);
        if (c->tab_host) (void)hipHostFree(c->tab_host);
        c->tab_dev = nullptr; c->tab_host = nullptr; c->tab_cap = 0;
        uint64_t cap = n < 1024 ? 1024 : n;
        HIP_TRY(hipMalloc(&c->tab_dev, cap * sizeof(ObjEntry)), "hipMalloc(batch table)");
        HIP_TRY(hipHostMalloc(&c->tab_host, cap * sizeof(ObjEntry), hipHostMallocDefault),
                "hipHostMalloc(batch table)");
        c->tab_cap = cap;
    }
    // Objects of size 0 contribute no tiles and no table entry.
    uint64_t m = 0;
    uint64_t ntiles[kTileShiftMax + 1] = {};
    for (uint64_t k = 0; k < n; ++k) {
        if (d[k].size == 0) continue;
        if (d[k].dst_off & 15u) return fail(S3DG_EINVAL, "dst_off must be a multiple of 16");
        const uint64_t nb = (d[k].size + kBlk - 1) / kBlk;
        ObjEntry &e = c->tab_host[m++];
        e.dst_off = d[k].dst_off;
        e.size = d[k].size;
        e.entropy = d[k].entropy;
        // XCD alignment: slot (mod 8) = 4 KiB granule (mod 8) of the block's address
        e.lead = (uint32_t)((((uintptr_t)dst_base + d[k].dst_off) >> 12) & 7);
        e.pad = 0;
        e.tile_begin = nb + e.lead;   // slot count until the tile size is known
        if (int r = make_prefix(nb, d[k].dedup, d[k].f_num, d[k].f_den, &e.pp)) return r;
        for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh)
            ntiles[sh] += (nb + e.lead + (1ull << sh) - 1) >> sh;
    }
    if (m == 0) return S3DG_OK;
    const uint32_t tshift = c->tile_shift ? c->tile_shift : pick_tile_shift(ntiles);
    uint64_t tiles = 0;
    for (uint64_t k = 0; k < m; ++k) {
        const uint64_t slots = c->tab_host[k].tile_begin;
        c->tab_host[k].tile_begin = tiles;
        tiles += (slots + (1ull << tshift) - 1) >> tshift;
    }
    hipStream_t s = (hipStream_t)stream;
    if (int r = tile_map_acquire(c, tiles, s)) return r;
    HIP_TRY(hipMemcpyAsync(c->tab_dev, c->tab_host, m * sizeof(ObjEntry), hipMemcpyHostToDevice, s),
            "hipMemcpyAsync(batch table)");
    HIP_TRY(hipEventRecord(c->tab_free, s), "hipEventRecord");
    HIP_TRY(launch_fill_batch(cfg_for(c, true), (uint8_t *)dst_base, c->tab_dev, m, tiles, tshift,
                              c->tile_obj, c->base_dev, s),
            "launch k_fill_batch");
    HIP_TRY(hipEventRecord(c->tile_free, s), "hipEventRecord");
    return S3DG_OK;
}

int s3dg_xoshiro_jump(uint64_t *state4, uint64_t n) {
    if (!state4) return fail(S3DG_EINVAL, "null state");
    uint64_t J[4];
    if (!jump_poly(n, J)) return fail(S3DG_EINVAL, "xoshiro characteristic polynomial unavailable");
    apply_jump(state4, J);
    return S3DG_OK;
}

// lanes per chunk + draws per lane for a chunk size; jump table cached per ctx
static int keystream_plan(s3dg_ctx *c, int mode, uint64_t chunk_bytes, uint64_t nchunks, KeystreamArgs &A,
                          const uint64_t **jtab) {
    const uint64_t nd = chunk_bytes / 8;
    // as many lanes per chunk as keep >= ks_min_draws draws per lane (the
    // jump costs 256 steps); up to 1024 lanes = 16 waves per chunk
    const uint64_t min_draws = c->ks_min_draws[mode];
    uint32_t lpc = 1;
    while (lpc < 1024 && nd / (2 * lpc) >= min_draws) lpc *= 2;
    // small launches (a few chunks): spread each chunk over more lanes, down
    // to 256 draws per lane, until the grid has ~4 waves per CU; otherwise a
    // 8 MiB request runs as 16 long waves and is latency-bound
    const uint64_t target_lanes = (uint64_t)c->cus * 4 * 64;
    while (lpc < 1024 && nchunks * lpc < target_lanes && nd / (2 * lpc) >= kKsMinSpan) lpc *= 2;
    uint64_t span = (nd + lpc - 1) / lpc;
    const uint64_t D = (uint64_t)c->ks[mode].draws;    // a lane stages D draws per iteration
    span = (span + D - 1) / D * D;
    if (span > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "chunk too large");
    A.lpc = lpc;
    A.span = (uint32_t)span;
    std::lock_guard<std::mutex> g(c->mu);
    const uint64_t key = ((uint64_t)lpc << 32) | span;
    auto it = c->jtabs.find(key);
    if (it == c->jtabs.end()) {
        std::vector<uint64_t> h(4 * (size_t)lpc, 0);
        for (uint32_t k = 0; k < lpc; ++k)
            if (!jump_poly((uint64_t)k * span, &h[4 * k]))
                return fail(S3DG_EINVAL, "xoshiro characteristic polynomial unavailable");
        uint64_t *d = nullptr;
        HIP_TRY(hipMalloc(&d, h.size() * 8), "hipMalloc(jump table)");
        HIP_TRY(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice), "hipMemcpy(jump table)");
        it = c->jtabs.emplace(key, d).first;
    }
    *jtab = it->second;
    return S3DG_OK;
}

int s3dg_xoshiro_fill(s3dg_ctx *c, void *dst, uint64_t len, uint64_t chunk_bytes,
                      uint64_t seed_base, void *stream) {
    CTX_SCOPE(c);
    if (len == 0) return S3DG_OK;
    if (chunk_bytes == 0 || (chunk_bytes & 127u))
        return fail(S3DG_EINVAL, "chunk_bytes must be a positive multiple of 128");
    if (!dst || !aligned16(dst)) return fail(S3DG_EINVAL, "dst must be a 16-byte aligned device pointer");
    KeystreamArgs A{};
    const uint64_t *jt = nullptr;
    if (int r = keystream_plan(c, 0, chunk_bytes, (len + chunk_bytes - 1) / chunk_bytes, A, &jt)) return r;
    A.nchunks = (len + chunk_bytes - 1) / chunk_bytes;
    A.chunk_bytes = chunk_bytes;
    A.obj_len = len;
    A.chunk0 = 0;
    A.seed_base = seed_base;
    A.seed_mode = 0;
    A.unique = 0xFFFFFFFFu;
    A.m_unique = 0;
    A.zf_num = 0;
    A.zf_den = 1;
    HIP_TRY(launch_keystream((uint8_t *)dst, A, jt, c->ks[0], (hipStream_t)stream), "launch k_keystream");
    return S3DG_OK;
}

int s3dg_internal_dgen_chunk(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride, uint64_t n_objs,
                             uint64_t blk_lo, uint64_t blk_hi, uint64_t dedup, uint32_t f_num,
                             uint32_t f_den, uint64_t seed_base, uint64_t first_obj, void *stream);

int s3dg_dgen_fill(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t blk_lo, uint64_t blk_hi,
                   uint64_t dedup, uint32_t f_num, uint32_t f_den, uint64_t seed, void *stream) {
    return s3dg_internal_dgen_chunk(c, dst, obj_size, 0, 1, blk_lo, blk_hi, dedup, f_num, f_den, seed, 0,
                                    stream);
}

// n_objs equal DG1 objects in one launch: blocks [blk_lo, blk_hi) of object
// first_obj + k at dst + k*stride, seeded object_entropy(seed_base, first_obj + k).
int s3dg_internal_dgen_chunk(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride, uint64_t n_objs,
                             uint64_t blk_lo, uint64_t blk_hi, uint64_t dedup, uint32_t f_num,
                             uint32_t f_den, uint64_t seed_base, uint64_t first_obj, void *stream) {
    CTX_SCOPE(c);
    if (obj_size == 0 || n_objs == 0) return S3DG_OK;
    const uint64_t nb = (obj_size + kDgenBlock - 1) / kDgenBlock;
    if (blk_hi > nb) blk_hi = nb;
    if (blk_lo >= blk_hi) return S3DG_OK;
    if (!dst || !aligned16(dst) || (stride & 15u)) return fail(S3DG_EINVAL, "dst and stride must be 16-byte aligned");
    const uint64_t span_bytes = (blk_hi * kDgenBlock < obj_size ? blk_hi * kDgenBlock : obj_size) - blk_lo * kDgenBlock;
    if (n_objs > 1 && stride < span_bytes) return fail(S3DG_EINVAL, "stride too small: objects overlap");
    if (f_den == 0 || f_num >= f_den) return fail(S3DG_EINVAL, "need f_num < f_den");
    if (nb > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "object larger than 2^32 blocks");
    KeystreamArgs A{};
    const uint64_t *jt = nullptr;
    if (int r = keystream_plan(c, 1, kDgenBlock, (blk_hi - blk_lo) * n_objs, A, &jt)) return r;
    const uint64_t U = s3dg_unique_blocks(nb, dedup);
    A.cpo = blk_hi - blk_lo;
    A.nchunks = A.cpo * n_objs;
    A.chunk_bytes = kDgenBlock;
    A.obj_len = obj_size;
    A.chunk0 = blk_lo;
    A.obj_stride = stride;
    A.seed_base = seed_base + (first_obj << 32);
    A.seed_step = 1ull << 32;
    A.seed_mode = 1;
    A.unique = U == nb ? 0xFFFFFFFFu : (uint32_t)U;
    A.m_unique = fastmod_magic(U == nb ? 1u : (uint32_t)U);
    A.zf_num = f_num;
    A.zf_den = f_den;
    HIP_TRY(launch_keystream((uint8_t *)dst, A, jt, c->ks[1], (hipStream_t)stream), "launch k_keystream(dgen)");
    return S3DG_OK;
}

int s3dg_crc32(s3dg_ctx *c, const void *dev, uint64_t len, void *stream, uint32_t *out) {
    CTX_SCOPE(c);
    if (!out || (len && !dev)) return fail(S3DG_EINVAL, "null argument");
    if (len && !aligned16(dev)) return fail(S3DG_EINVAL, "dev must be 16-byte aligned");
    std::lock_guard<std::mutex> g(c->crc_mu);
    HIP_TRY(crc32_device((const uint8_t *)dev, len, (hipStream_t)stream, out, &c->crc_tab, &c->crc_seg,
                         &c->crc_seg_cap),
            "crc32 kernel");
    return S3DG_OK;
}

int s3dg_internal_crc_device(s3dg_ctx *c, const void *dev, uint64_t len, void *stream, uint32_t *out) {
    return s3dg_crc32(c, dev, len, stream, out);
}

uint32_t s3dg_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return crc32_combine(crc1, crc2, len2);
}

uint32_t s3dg_crc32_host(uint32_t crc, const uint8_t *p, uint64_t n) {
    return crc32_host_update(crc, p, n);
}

int s3dg_write_ceiling(s3dg_ctx *c, void *dst, uint64_t len, uint32_t pattern, void *stream) {
    CTX_SCOPE(c);
    if (!dst || !aligned16(dst) || (len % kBlk))
        return fail(S3DG_EINVAL, "dst must be 16-byte aligned and len a multiple of 4096");
    HIP_TRY(launch_write_ceiling(cfg_for(c), (uint8_t *)dst, len, pattern, nullptr, 0, (hipStream_t)stream),
            "launch k_write_ceiling");
    return S3DG_OK;
}

int s3dg_write_ceiling_tiled(s3dg_ctx *c, void *dst, uint64_t len, uint32_t pattern, void *stream) {
    CTX_SCOPE(c);
    if (!dst || !aligned16(dst) || (len % kBlk))
        return fail(S3DG_EINVAL, "dst must be 16-byte aligned and len a multiple of 4096");
    if (len == 0) return S3DG_OK;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t nthr = (len / kBlk + 63) / 64;
    std::lock_guard<std::mutex> g(c->mu);
    if (int r = tile_map_acquire(c, nthr, s)) return r;
    HIP_TRY(launch_write_ceiling(cfg_for(c, true), (uint8_t *)dst, len, pattern, c->tile_obj, nthr, s),
            "launch k_write_ceiling(tiled)");
    HIP_TRY(hipEventRecord(c->tile_free, s), "hipEventRecord");
    return S3DG_OK;
}

int s3dg_device_alloc(s3dg_ctx *c, uint64_t bytes, void **out) {
    CTX_SCOPE(c);
    if (!out) return fail(S3DG_EINVAL, "null output");
    HIP_TRY(hipMalloc(out, bytes), "hipMalloc");
    return S3DG_OK;
}

int s3dg_device_free(s3dg_ctx *c, void *p) {
    CTX_SCOPE(c);
    HIP_TRY(hipFree(p), "hipFree");
    return S3DG_OK;
}

int s3dg_host_alloc_pinned(uint64_t bytes, void **out) {
    if (!out) return fail(S3DG_EINVAL, "null output");
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocDefault), "hipHostMalloc");
    return S3DG_OK;
}

int s3dg_host_free_pinned(void *p) {
    HIP_TRY(hipHostFree(p), "hipHostFree");
    return S3DG_OK;
}

int s3dg_d2h_async(s3dg_ctx *c, void *host, const void *dev, uint64_t len, void *stream) {
    CTX_SCOPE(c);
    HIP_TRY(hipMemcpyAsync(host, dev, len, hipMemcpyDeviceToHost, (hipStream_t)stream),
            "hipMemcpyAsync(D2H)");
    return S3DG_OK;
}

int s3dg_h2d_async(s3dg_ctx *c, void *dev, const void *host, uint64_t len, void *stream) {
    CTX_SCOPE(c);
    HIP_TRY(hipMemcpyAsync(dev, host, len, hipMemcpyHostToDevice, (hipStream_t)stream),
            "hipMemcpyAsync(H2D)");
    return S3DG_OK;
}

int s3dg_stream_create(s3dg_ctx *c, void **out) {
    CTX_SCOPE(c);
    if (!out) return fail(S3DG_EINVAL, "null output");
    hipStream_t s;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    *out = (void *)s;
    return S3DG_OK;
}

int s3dg_stream_destroy(s3dg_ctx *c, void *stream) {
    CTX_SCOPE(c);
    HIP_TRY(hipStreamDestroy((hipStream_t)stream), "hipStreamDestroy");
    return S3DG_OK;
}

int s3dg_sync(s3dg_ctx *c, void *stream) {
    CTX_SCOPE(c);
    if (stream) HIP_TRY(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
    else HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return S3DG_OK;
}

}  // extern "C"

// ---- host-buffer drop-ins ----------------------------------------------------

namespace {

struct DefaultCtx {
    std::mutex mu;
    s3dg_ctx *ctx = nullptr;
    // base blocks in HBM, each uploaded once: A_BASE_BLOCK (random, once per
    // process, src/constants.rs:715-720), BASE_BLOCK (:725-729), and the
    // caller's block of a seeded call (re-uploaded per call; calls are
    // serialised by `mu` and each drains its streams before returning)
    void *base_proc = nullptr, *base_proc2 = nullptr, *base_user = nullptr;
    void *scratch[2] = {nullptr, nullptr};
    hipStream_t st[2] = {nullptr, nullptr};
    static constexpr uint64_t kChunk = 64ull << 20;   // 64 MiB per device chunk
};

DefaultCtx &dflt() {
    static DefaultCtx *d = new DefaultCtx();   // intentionally leaked: outlives atexit
    return *d;
}

int random_bytes(uint8_t *dst, size_t n);

int dflt_init(DefaultCtx &D) {
    if (D.ctx) return S3DG_OK;
    int dev = 0;
    if (const char *e = getenv("S3DLIO_GPU_DEVICE")) dev = atoi(e);
    s3dg_ctx *c = nullptr;
    if (int r = s3dg_ctx_create(dev, &c)) return r;
    for (int k = 0; k < 2; ++k) {
        HIP_TRY(hipMalloc(&D.scratch[k], DefaultCtx::kChunk), "hipMalloc(scratch)");
        HIP_TRY(hipStreamCreateWithFlags(&D.st[k], hipStreamNonBlocking), "hipStreamCreate");
    }
    uint8_t b[kBlk];
    HIP_TRY(hipMalloc(&D.base_user, kBlk), "hipMalloc(base block)");
    HIP_TRY(hipMalloc(&D.base_proc, kBlk), "hipMalloc(base block)");
    if (int r = random_bytes(b, kBlk)) return r;
    HIP_TRY(hipMemcpy(D.base_proc, b, kBlk, hipMemcpyHostToDevice), "hipMemcpy(base block)");
    HIP_TRY(hipMalloc(&D.base_proc2, kBlk), "hipMalloc(base block)");
    if (int r = random_bytes(b, kBlk)) return r;
    HIP_TRY(hipMemcpy(D.base_proc2, b, kBlk, hipMemcpyHostToDevice), "hipMemcpy(base block)");
    D.ctx = c;
    return S3DG_OK;
}

// Generate into a host buffer through two 64 MiB device chunks on two
// streams, so chunk k+1's kernel overlaps chunk k's D2H copy.  `pp` selects
// the layout (controlled, or f_den = 0: generate_random_data's); `base` is
// the device base block.
int fill_host(DefaultCtx &D, uint8_t *buf, uint64_t len, const PrefixParams &pp, uint64_t entropy,
              const void *base) {
    CTX_SCOPE(D.ctx);     // the calling thread may have another device current
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    const uint64_t cb = DefaultCtx::kChunk / kBlk;
    for (uint64_t b0 = 0, k = 0; b0 < nb; b0 += cb, ++k) {
        const uint64_t b1 = b0 + cb < nb ? b0 + cb : nb;
        const int sl = (int)(k & 1);
        HIP_TRY(launch_fill_stream(cfg_for(D.ctx), (uint8_t *)D.scratch[sl], len, 0, 1, (uint32_t)b0,
                                   (uint32_t)b1, entropy, 0, pp, base, D.st[sl]),
                "launch k_fill_stream(host chunk)");
        const uint64_t off = b0 * kBlk;
        const uint64_t n = (b1 * kBlk < len ? b1 * kBlk : len) - off;
        HIP_TRY(hipMemcpyAsync(buf + off, D.scratch[sl], n, hipMemcpyDeviceToHost, D.st[sl]),
                "hipMemcpyAsync(D2H)");
    }
    HIP_TRY(hipStreamSynchronize(D.st[0]), "hipStreamSynchronize");
    HIP_TRY(hipStreamSynchronize(D.st[1]), "hipStreamSynchronize");
    return S3DG_OK;
}

int fill_host_controlled(DefaultCtx &D, uint8_t *buf, uint64_t len, uint64_t dedup, uint64_t compress,
                         uint64_t entropy, const void *base) {
    uint32_t fn, fd;
    if (int r = s3dg_compress_ratio(compress, &fn, &fd)) return r;
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    PrefixParams pp;
    if (int r = make_prefix(nb, dedup, fn, fd, &pp)) return r;
    return fill_host(D, buf, len, pp, entropy, base);
}

// generate_random_data layout (seeded analogue) into a host buffer; block i
// seeded entropy + i.
int fill_host_random(DefaultCtx &D, uint8_t *buf, uint64_t len, uint64_t entropy, const void *base) {
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    if (nb > 0xFFFFFFFFull) return fail(S3DG_EINVAL, "object larger than 2^32 blocks");
    PrefixParams pp{};
    pp.unique = 0xFFFFFFFFu;
    pp.f_den = 0;
    pp.m_unique = fastmod_magic(1);
    pp.m_fden = fastmod_magic(1);
    return fill_host(D, buf, len, pp, entropy, base);
}

int random_bytes(uint8_t *dst, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t k = getrandom(dst + got, n - got, 0);
        if (k <= 0) return fail(S3DG_EINVAL, "getrandom failed");
        got += (size_t)k;
    }
    return S3DG_OK;
}

uint64_t time_entropy() {      // SystemTime::now() ... as_nanos() as u64, :192-195
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

}  // namespace

extern "C" {

int s3dg_internal_fail(int code, const char *msg) { return fail(code, msg); }

s3dg_ctx *s3dg_internal_default_ctx(int *err) {
    DefaultCtx &D = dflt();
    std::lock_guard<std::mutex> g(D.mu);
    const int r = dflt_init(D);
    if (err) *err = r;
    return r ? nullptr : D.ctx;
}

// generate_random_data payload for generate_object: seeded (ctx default base
// block, entropy = seed) or unseeded (time entropy + per-process BASE_BLOCK).
int s3dg_internal_random_host(uint8_t *buf, uint64_t len, uint64_t entropy, int use_process_base) {
    if (len == 0) return S3DG_OK;
    DefaultCtx &D = dflt();
    std::lock_guard<std::mutex> g(D.mu);
    if (int r = dflt_init(D)) return r;
    if (!use_process_base) return fill_host_random(D, buf, len, entropy, D.ctx->base_dev);
    return fill_host_random(D, buf, len, time_entropy(), D.base_proc2);
}

int s3dlio_generate_random_data(uint8_t *buf, size_t size) {
    if (size == 0) return S3DG_OK;
    if (!buf) return fail(S3DG_EINVAL, "null buffer");
    return s3dg_internal_random_host(buf, size, 0, 1);
}

int s3dlio_fill_controlled_data(uint8_t *buf, size_t len, size_t dedup, size_t compress) {
    if (len == 0) return S3DG_OK;
    if (!buf) return fail(S3DG_EINVAL, "null buffer");
    DefaultCtx &D = dflt();
    std::lock_guard<std::mutex> g(D.mu);
    if (int r = dflt_init(D)) return r;
    return fill_host_controlled(D, buf, len, dedup, compress, time_entropy(), D.base_proc);
}

int s3dlio_fill_controlled_data_seeded(uint8_t *buf, size_t len, size_t dedup, size_t compress,
                                       uint64_t entropy, const uint8_t *base4096) {
    if (len == 0) return S3DG_OK;
    if (!buf) return fail(S3DG_EINVAL, "null buffer");
    DefaultCtx &D = dflt();
    std::lock_guard<std::mutex> g(D.mu);
    if (int r = dflt_init(D)) return r;
    const void *base = D.ctx->base_dev;
    if (base4096) {
        CTX_SCOPE(D.ctx);
        HIP_TRY(hipMemcpy(D.base_user, base4096, kBlk, hipMemcpyHostToDevice), "hipMemcpy(base block)");
        base = D.base_user;
    }
    return fill_host_controlled(D, buf, len, dedup, compress, entropy, base);
}

}  // extern "C"
