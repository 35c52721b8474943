// s3dg_internal.h — shared between the HIP kernels and the C-ABI layer.
#pragma once
#include <sched.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "s3dlio_gpu.h"

extern "C" int s3dg_internal_fail(int code, const char *msg);
struct s3dg_ctx;

namespace s3dg {

constexpr uint32_t kBlk = 4096;   // BLK_SIZE   src/constants.rs:326
constexpr uint32_t kHalf = 2048;  // HALF_BLK   src/constants.rs:329
constexpr uint32_t kMod = 32;     // MOD_SIZE   src/constants.rs:352
constexpr uint64_t kDgenBlock = 1ull << 20;   // DGEN_BLOCK_SIZE src/constants.rs:348
// batch tiles (tile -> object map granule) are 2^tshift blocks, tshift in
// [kTileShiftMin, kTileShiftMax], chosen per launch (s3dg_capi.cpp pick_tile_shift)
constexpr uint32_t kTileShiftMin = 1, kTileShiftMax = 6;
// the per-launch choice considers 8..64-block tiles only: 2- and 4-block tiles
// (s3dg_set_batch_tile) cut dead slots but lose more to records, e.g. 16-B
// packed 20 KiB objects 2556 vs 2917 GB/s (profiles/r02/diag/desc40/ab3_*.log)
constexpr uint32_t kTileShiftAutoMin = 3;
// tshift 0 (one record per 4 KiB granule of the batch's address range, no
// per-object lead) is the dense layout for small packed objects
constexpr int kWavesPerWG = 4;

// Zero-prefix parameters of one object: const_len(u) =
//   floor_len + ((u+1)*rem)/f_den - (u*rem)/f_den   (closed form of the
// accumulator at src/data_gen.rs:174-190; rem < f_den).
struct PrefixParams {
    uint32_t unique;     // U, src/data_gen.rs:162-167 (0xFFFFFFFF: U == nblocks, u = i)
    uint32_t floor_len;
    uint32_t rem;
    uint32_t f_den;      // 0: generate_random_data block layout (src/data_gen.rs:102-132)
    uint64_t m_unique;   // Lemire fastmod constants: floor(2^64 / d) + 1
    uint64_t m_fden;
};

// a % d for 32-bit a and d >= 1 with M = fastmod_magic(d) (Lemire, Kaser &
// Kurz 2019, "Faster remainder by direct computation"); exact for all a, d < 2^32.
inline uint64_t fastmod_magic(uint32_t d) { return ~0ull / d + 1; }

// Batch sub-batches reach the device as the caller's 40-B descriptors
// (empty objects dropped); the record ranges are derived there:
// tile layouts by an exclusive scan of the objects' tile counts
// (launch_batch_scan, s3dg_batch.hip), the dense layout from each object's
// granule and its successor's (k_batch_map).
static_assert(sizeof(s3dg_obj_desc) == 40, "s3dg_obj_desc is 40 bytes");

// One tile (2^tshift slots) of a batch object, written by k_batch_map /
// k_tile_map_uniform so the fill
// kernel reaches everything with a single 64-byte scalar load.
struct TileRec {
    uint64_t dst_off;      // byte offset of the object
    uint64_t size;         // object size
    uint64_t entropy;
    uint32_t first;        // first slot of the tile: tile index x tile blocks
    uint32_t lead;         // slot of block 0: block = first + slot - lead
    PrefixParams pp;
};
static_assert(sizeof(TileRec) == 64, "TileRec is one s_load_dwordx16");


// store cache policy of the fill kernels (s3dg_set_store_policy)
constexpr int kStorePlain = 0, kStoreNT = 1, kStoreSC1 = 2, kStoreNTSC1 = 3;

struct LaunchCfg {
    int store;             // kStorePlain / kStoreNT / kStoreSC1 / kStoreNTSC1
    int waves_per_block;   // 1, 2 or 4 wave64s per 4 KiB block (one workgroup)
    uint32_t dyn_lds = 0;  // reserved dynamic LDS per workgroup (occupancy cap)
    uint32_t prefetch_tiles = 0;   // batch: tile-record prefetch distance (0 = off)
    uint32_t pace = 0;             // store-only reference only: wave-0 delay before the stores
    uint32_t rt_floor = 0;         // batch kernel: wall-clock ticks (10 ns) from workgroup start to its stores
};

// Dynamic LDS that caps a fill launch at `wgs` resident workgroups per CU
// (0 = no cap).  Static LDS of the fill kernels: one BlockLds per block.
uint32_t occupancy_lds(int wgs, uint32_t static_lds);
constexpr uint32_t kFillStaticLds = kBlk + 16;
hipError_t fill_occupancy(const LaunchCfg &lc, bool batch, int *wgs_per_cu);

hipError_t launch_fill_stream(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size,
                              uint64_t stride, uint64_t n_objs, uint32_t blk_lo,
                              uint32_t blk_hi, uint64_t seed_base, uint64_t first_obj,
                              PrefixParams pp, const void *base_dev, hipStream_t s);

// Batch records built on the device from the uploaded descriptors (the scan,
// then k_batch_map: prefix parameters per object and its records), then
// k_fill_batch over total_recs << tshift slots.
// Sub-batch records from its n non-empty descriptors d (device): tile
// layouts (tshift >= kTileShiftMin) read rec_lo[k] = the exclusive scan of
// the tile counts; the dense layout (tshift 0) places object k's block 0 at
// slot lead0 + (d[k].dst_off - first_off) / 4 KiB.
hipError_t launch_batch_map(const s3dg_obj_desc *d, uint64_t n, const uint64_t *rec_lo, TileRec *tiles,
                            uint32_t tshift, uintptr_t base, uint64_t lead0, uint64_t first_off, hipStream_t s);
// rec_lo[k] = sum of tiles(d[j]) for j < k, tiles(o) = (blocks + lead + 2^tshift - 1) >> tshift,
// lead = ((base + o.dst_off) >> 12) & 7.  tmp == nullptr: *tmp_bytes = the scratch size n needs.
hipError_t launch_batch_scan(const s3dg_obj_desc *d, uint64_t n, uint32_t tshift, uintptr_t base, uint64_t *rec_lo,
                             void *tmp, size_t *tmp_bytes, hipStream_t s);
hipError_t launch_batch_tiles(const LaunchCfg &lc, uint8_t *dst_base, uint64_t total_tiles, uint32_t tshift,
                              TileRec *tiles, const void *base_dev, hipStream_t s);

// A uniform stream through the batch kernel: records built on the device
// (k_tile_map_uniform), then k_fill_batch.
hipError_t launch_fill_uniform_tiles(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size, uint64_t stride,
                                     uint64_t n_objs, uint32_t tiles_per_obj, uint32_t tshift, uint32_t lead,
                                     uint64_t ent0, PrefixParams pp, TileRec *tiles, const void *base_dev,
                                     hipStream_t s);

// The store-only reference of the same launch (s3dg_write_ceiling_fill).
hipError_t launch_fill_uniform_tiles_ablated(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size, uint64_t stride,
                                             uint64_t n_objs, uint32_t tiles_per_obj, uint32_t tshift, uint32_t lead,
                                             PrefixParams pp, TileRec *tiles, const void *base_dev, hipStream_t s);

// K2 keystream launch: chunks [chunk0, chunk0 + nchunks) of an obj_len-byte
// object, chunk k at dst + (k - chunk0) * chunk_bytes.
struct KeystreamArgs {
    uint64_t nchunks;       // chunks in this launch
    uint64_t chunk_bytes;
    uint64_t obj_len;       // object size (sets the ragged last chunk)
    uint64_t chunk0;        // first chunk index
    uint64_t seed_base;
    uint32_t seed_mode;     // 0: seed_base + k (npz.rs:381); 1: seed_base ^ ((k % U) * phi) (dgen mode)
    uint32_t unique;        // U for seed_mode 1 (0xFFFFFFFF: none)
    uint64_t m_unique;      // fastmod constant for U
    uint64_t zf_num, zf_den;  // zero prefix = floor(chunk_len * zf_num / zf_den)
    uint32_t lpc, span;     // lanes per chunk, draws per lane
    // several objects per launch: chunk c -> object c / cpo (0 = one object),
    // its chunk chunk0 + c % cpo, written at dst + object*obj_stride, seeded
    // seed_base + object*seed_step
    uint64_t cpo, obj_stride, seed_step;
    // workgroups per XCD group (power of two; 1 = the dispatcher's round-robin
    // dealing): each full group of 8*xg workgroups is remapped so the xg
    // workgroups one XCD receives take xg adjacent work units
    uint32_t xg;
    // set by launch_keystream: workgroups of the static grid; for a persistent
    // launch (ks_ctr given, more than one round of resident waves) the stream's
    // two sets of 8 queue counters (KsCounters) and the set this launch uses
    uint32_t nwg;
    uint32_t par;
    uint64_t *ctr;
    // first draw of every chunk the launch covers (lane sub starts at draw
    // z0 + sub*span; jtab[sub] = x^(z0 + sub*span)): a DG1 launch over the
    // chunks' tails whose zero prefixes k_zero_prefix has written
    uint64_t z0;
    // byte offset of this argument set's first chunk from the kernel's dst
    // (the tail set of a persistent launch, below)
    uint64_t doff;
};

// DG1 zero prefixes in the fill's store shape (paired with a keystream launch
// over the tails, A.z0 > 0): the first zw bytes (a multiple of 16) of each
// of nchunks chunks (chunk c of object c / cpo at dst + (c / cpo)*obj_stride +
// (c % cpo)*chunk_bytes) set to zero; one workgroup of 64 x lc.waves_per_block
// threads per 4 KiB granule, lc.store, lc.dyn_lds capping the resident workgroups.
hipError_t launch_zero_prefix(uint8_t *dst, uint64_t nchunks, uint64_t cpo, uint64_t obj_stride, uint64_t chunk_bytes,
                              uint32_t zw, const LaunchCfg &lc, hipStream_t s);

// Per-stream queue counters of persistent keystream launches: 2 sets x 8
// counters, 128 B apart (kKsCtrBytes, zeroed at allocation); `par` alternates
// per persistent launch, each launch zeroing the other set for the next.
constexpr size_t kKsCtrBytes = 2 * 8 * 128;
struct KsCounters {
    uint64_t *dev = nullptr;
    uint32_t par = 0;
};

// k_keystream launch shape: draws staged per lane per iteration (16, 32, 64),
// waves per workgroup (1, 2, 4), resident workgroups per CU cap (0 = none),
// store cache policy.
struct KsShape {
    int draws, waves, wgs_per_cu;
    int store;             // kStorePlain / kStoreNT / kStoreSC1 / kStoreNTSC1
    int xcd_waves;         // adjacent waves per XCD group (power of two; <= waves: dealing order)
};
// ctrs: the stream's queue counters (persistent launches), or null for the
// static grid.  cus: compute units of the device.  persist_rounds: launches
// of at least that many rounds of resident waves run persistent (0: never;
// negative: the default rule, 1-wave workgroups from kKsPersistRounds).
// tail / tail_jtab: a second argument set (other lanes per chunk, A2.doff)
// whose units a persistent launch hands out after A's, so the launch ends on
// shorter units; a static-grid launch runs it as a second launch.
hipError_t launch_keystream(uint8_t *dst, const KeystreamArgs &A, const uint64_t *jtab,
                           const KsShape &sh, hipStream_t s, KsCounters *ctrs = nullptr, int cus = 0,
                           int persist_rounds = -1, const KeystreamArgs *tail = nullptr,
                           const uint64_t *tail_jtab = nullptr);
hipError_t keystream_occupancy(const KsShape &sh, int *wgs_per_cu);

// thr/nthr: records for the tiled shape's trailing loads (lc.prefetch_tiles), or null
hipError_t launch_write_ceiling(const LaunchCfg &lc, uint8_t *dst, uint64_t len,
                                uint32_t pattern, const TileRec *thr, uint64_t nthr, hipStream_t s);


// ---- context internals (s3dg_capi.cpp) ---------------------------------------
// Zero-prefix parameters of an object of nblocks 4 KiB blocks
// (src/data_gen.rs:162-190); S3DG_EINVAL on a bad ratio.
int make_prefix(uint64_t nblocks, uint64_t dedup, uint32_t f_num, uint32_t f_den, PrefixParams *pp);
// generate_random_data's block layout (f_den = 0, src/data_gen.rs:102-132)
PrefixParams random_layout_prefix();
LaunchCfg ctx_stream_cfg(const s3dg_ctx *c);   // the context's stream-kernel launch knobs
const void *ctx_base(const s3dg_ctx *c);       // the context's 4 KiB base block in HBM

// ---- host-buffer engine (s3dg_host.cpp) --------------------------------------
// Pinned host allocations made by this library (s3dg_host_alloc_pinned[_local]
// and the engine's own bounce buffers and rings): the only host memory a
// kernel may store into directly.  pinned_owned: [p, p+n) lies inside one.
void pinned_register(const void *p, uint64_t n);
void pinned_unregister(const void *p);
bool pinned_owned(const void *p, uint64_t n);
// hipHostMalloc from a thread bound to the device's local CPUs (its NUMA node).
hipError_t host_alloc_pinned_local(int device, uint64_t bytes, void **out);

// Staging set of a host slot: two 64 MiB device chunks, two streams and a
// 4 KiB device block for a caller's base block; for small calls a pinned
// bounce buffer the kernels write straight into (no copy engine) and the
// events that hand its pieces to the calling thread (lazily).
constexpr int kSmallPieces = 8;
struct HostStaging {
    int slot = 0;
    void *buf[2] = {nullptr, nullptr};
    hipStream_t st[2] = {nullptr, nullptr};
    void *base_user = nullptr;
    uint8_t base_user_host[4096];        // the caller's block last uploaded to base_user
    bool base_user_valid = false;
    void *pin[2] = {nullptr, nullptr};   // pinned bounce buffers (staged D2H mode only, lazily)
    uint8_t *bounce = nullptr;           // pinned, small calls (lazily)
    uint64_t bounce_bytes = 0;
    hipEvent_t ev[kSmallPieces] = {};
};
// What to generate into host memory: the fill_controlled_data / random-data
// layouts (4 KiB blocks, pp) or DG1 (dgen = true, 1 MiB blocks).
struct HostJob {
    enum Base { kBaseCtx, kBaseProcA, kBaseProcB, kBaseUser };
    bool dgen = false;
    uint64_t obj_len = 0;
    uint64_t entropy = 0;          // block seeds u + entropy; DG1: the seed
    PrefixParams pp{};
    Base base = kBaseCtx;
    const uint8_t *user_base = nullptr;
    uint64_t dedup = 1;            // DG1
    uint32_t f_num = 0, f_den = 1; // DG1
};
int host_slot_count(int *n);
int host_next_slot(int *slot);     // round-robin
int host_staging_acquire(int slot, HostStaging **out);
void host_staging_release(HostStaging *sg);   // waits for its streams
int host_run(HostStaging *sg, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n);
int host_run_split(HostStaging *sg0, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n);
// Launch the job's generation blocks [b_lo, b_hi) (4 KiB or, DG1, 1 MiB
// units) at dst (device or library-pinned host memory) on stream st of the
// staging set's slot; the caller's base block must already be in place.
int host_launch_blocks(HostStaging *sg, const HostJob &J, uint8_t *dst, uint64_t b_lo, uint64_t b_hi,
                       hipStream_t st);

// Read-ahead ring of a streaming generator (s3dg_generator.cpp): 2 halves of
// `half` bytes of pinned host memory on the slot's NUMA node, written by the
// keystream kernel directly, one event per half.  Pooled per slot; at most
// kMaxRings exist at once (host_ring_acquire then returns S3DG_OK with *out
// null and the generator uses the synchronous path).
struct HostRing {
    int slot = 0;
    uint64_t half = 0;
    uint8_t *mem = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
};
int host_ring_acquire(int slot, uint64_t half, HostRing **out);
void host_ring_release(HostRing *r);   // the caller has waited for its pending halves

// ---- CRC-32 (s3dg_crc.hip) -------------------------------------------------
uint32_t crc32_host_update(uint32_t crc, const uint8_t *p, uint64_t n);
uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

// nseg equal segments of seg_len bytes at seg_stride: whole 1 KiB rows are
// hashed on the device (nreg regions of `rows` rows), the < 1 KiB tail of
// each segment on the host.
struct CrcSegPlan {
    uint64_t nseg, seg_len, seg_stride, seg_rows, regs_per_seg, nreg;
    uint32_t rows;
};
hipError_t crc_tables_device(void **tab_cache);
CrcSegPlan crc_seg_plan(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride);
hipError_t crc_seg_launch(const CrcSegPlan &P, const uint8_t *dev, void *tab_dev, uint32_t *out_dev,
                          hipStream_t s);
void crc_seg_fold(const CrcSegPlan &P, const uint32_t *regions, const uint8_t *const *tails,
                  uint32_t *crcs);

// ---- NUMA placement of host buffers (s3dg_numa.cpp) -------------------------
bool device_local_cpus(int device, cpu_set_t *out);
int device_numa_node(int device);   // -1 when unknown
// Binds the calling thread to the device's local CPUs for its lifetime (no-op
// when sysfs has no answer or the affinity mask already lies inside them).
class NumaScope {
public:
    explicit NumaScope(int device);
    ~NumaScope();
    NumaScope(const NumaScope &) = delete;
    NumaScope &operator=(const NumaScope &) = delete;
private:
    cpu_set_t saved_;
    bool active_ = false;
};

// Makes `device` current for the scope and restores the caller's current
// device afterwards, so a C-ABI call never changes the calling thread's HIP
// (and torch's) current device.
struct DeviceScope {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
        else prev = -1;                                  // nothing to restore
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    bool ok() const { return err == hipSuccess; }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};

}  // namespace s3dg
