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

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <memory>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

using namespace s3dg;

#ifndef S3DG_DIAG_OLDTILECOST
#define S3DG_DIAG_OLDTILECOST 0   // diagnostic builds only: the first cost model's tile size (A/B)
#endif
constexpr int kDefaultOccStream = 14, kDefaultOccBatch = -1;   // batch: -1 = per launch (below)
// Batch-kernel occupancy per launch: uncapped (32
// resident 1-wave workgroups per CU) unless the launch's zero prefixes end on
// a 64-B line (compress c with 64 % c == 0: c = 2, 4, 8, ... and ratios such
// as 4/3), where a cap of 29 resident workgroups writes 3-7 % faster: config 3
// 7214-7260 -> 7416-7424 GB/s, d1 c4 6925 -> 7435, d1 c8 6933 -> 7436, while
// the same cap costs c = 1, 1.5 and 3 (mid-line prefixes) 2-4 %
// (profiles/r03/diag/cfg3/power/).
// The target passed to occupancy_lds: asking for 30 gives a 5632-B LDS
// footprint, i.e. 29 resident (no 512-B granule gives exactly 30), which is
// what was measured and what s3dg_query_occupancy(ctx, 2, ..) reports.
constexpr int kOccZeroLines = 30;
// Zero prefixes of at least half the block that end inside a line (c = 3,
// 5, 6, 7, ...): uncapped, with the stores held until 100 wall-clock ticks
// (1 us) after the workgroup starts, whatever the GFX clock (DESIGN.md
// §5.1.2: config 5 7343 -> 7535-7540 GB/s, d1 c3 7115-7181 -> 7407-7450;
// config 2 would lose 0.4 %, so prefix-free launches keep no floor).
constexpr int kDefaultBatchRtFloor = -1;   // per launch
// Mixed-size batches (BASELINE config 4): one tile size per launch leaves the
// last tile of every object ragged, and small objects (a few blocks in a
// 64-block tile) are mostly dead slots.  Objects below kDefaultSplitBlocks
// blocks get a launch of their own, whose tile size is picked for them
// (DESIGN.md §5.1); 0 = off.
constexpr uint32_t kDefaultSplitBlocks = 0;
constexpr uint32_t kRtFloorMidZeros = 100;
// Uniform streams of large objects without a zero prefix (config 2): the same
// 1 us store floor.  On some boxes 10-45 % of such launches run 12.1-12.9 ms
// instead of 11.0-11.2 (round 4's driver line; round 5's final and lab boxes,
// at the normal clock and power): with the floor those boxes ran 0 % and
// 0-30 % slow launches, +1.0 / +1.9 % by mean (tools/dip_lab.py, bench.py
// --pace A/Bs, profiles/r05/dip/), while a box without them lost 0.2 %.
// Small objects (config 8) and batches (config 4) showed few slow launches
// and no gain (0 / -0.7 %), so they keep no floor.  DESIGN.md §5.1.4.
constexpr uint32_t kRtFloorLargeUniform = 100;
constexpr uint64_t kRtFloorLargeBlocks = 512;   // objects of >= 2 MiB
// Launch classes by zero prefix (per launch; batches by majority of blocks)
enum ZeroClass { kZcNone = 0, kZcLines = 1, kZcMidHeavy = 2 };
// The mid-line class's store floor is checked by measurement (round 4).  It
// won 2.6 % on one box and lost 0.5-1.6 % to a plain launch on four others
// (DESIGN.md §5.1.2): it compensates for the chip's power state, which
// differs between boxes.  So a context times its own large launches of that
// class (HIP events around the fill, read back without waiting, at a later
// launch) and runs the floor or the plain uncapped launch, whichever wrote
// faster: after kTuneFirst launches of each (alternating; the context's first
// timed launch is a warm-up and is not sampled), the MEANS of each one's last
// kTuneKeep rates, the plain launch taken only when it beats the current
// choice's mean by more than kTuneMargin (the class setting otherwise), so two
// candidates within the noise of each other do not flip from run to run
// (the best-of-3 rule did).  Means, not medians (round
// 6): on a box with the slow mode 47 % of plain config-5 launches ran 12.1-12.8
// ms against 11.0-11.3, which a median of five does not see, so the tuner kept
// probing a candidate 4 % slower by mean (tools/dip_lab.py,
// profiles/r06/slow/).  The loser is probed again after kTuneReprobe launches,
// and each probe that confirms the choice doubles that interval (up to
// kTuneReprobeMax), so a settled choice costs few probe launches.
// The line-aligned class keeps its cap unmeasured: it won 4-9 % on every box.
// Launches below kTuneMinBytes use the current choice; an explicit
// s3dg_set_occupancy / s3dg_set_batch_pace (or S3DG_ZC_TUNE=0) turns the
// check off.
constexpr uint64_t kTuneMinBytes = 1ull << 30;
constexpr uint64_t kTuneReprobe = 32, kTuneReprobeMax = 1024;
constexpr int kTuneKeep = 5, kTuneFirst = 4;
constexpr double kTuneMargin = 0.01;
struct ZcTuner {
    int best = 0;                  // 0 = the fitted rule, 1 = uncapped, no floor
    uint64_t launches = 0;         // timed launches issued
    uint64_t issued[2] = {0, 0};
    uint64_t interval = kTuneReprobe;   // launches between probes of the loser
    uint64_t next_probe = 0;            // launch index of the next probe (0: not scheduled)
    bool warm = false;                  // the first timed launch has been dropped
    double recent[2][kTuneKeep] = {};   // GB/s of the last kTuneKeep timed launches of each
    int samples[2] = {0, 0};
    struct Pending {
        hipEvent_t a, b;
        double bytes;
        int cand;
    };
    std::vector<Pending> pend;
    std::vector<hipEvent_t> spare;
};
constexpr uint32_t kDefaultPrefetch = 256;   // in 64-block units; > resident workgroups / 64
constexpr int kDefaultStreamTiles = 1;
constexpr uint64_t kStreamTilesMinBlocks = 16384;   // smaller streams: 2D kernel, no tile-map launch
constexpr int kDefaultStoreStream = kStoreNTSC1, kDefaultStoreBatch = kStoreSC1;
// dense batch layouts (one 64-B record per 4 KiB block): nt sc1 stores keep
// the written lines out of L2, where sc1 evicts the prefetched records
// (tools/batch_lab.py, profiles/r02/diag/batch_lab_store_*: 20 KiB+5 objects 4766 -> 6092 GB/s,
// dense 32 KiB 5977 -> 6663, dense 64 KiB 5992 -> 6472; tiled layouts keep sc1)
constexpr int kDefaultStoreDense = kStoreNTSC1;
// Draws per lane (npz keystream, DG1).  Since the jump's state sequence runs
// on the scalar unit (k_keystream), longer lanes win: 2048 draws per lane
// (K2 8 GiB launches 6096 -> 6621 GB/s, 80 GiB 6436 -> 6596; DG1 c1 6141 ->
// 6604 / 6434 -> 6621; profiles/r02/diag/ks/ks_draws_sweep.log), and K2
// launches of at least kKsLongRounds rounds of resident waves take 4096
// (80 GiB: 6718; with 1-wave workgroups in XCD groups also 8 GiB launches,
// profiles/r02/diag/ks/ks_draws_new_shape.log).  DG1 stays at 2048:
// at 4096 a wave would span two 1 MiB blocks and lose the scalar jump.
constexpr uint64_t kDefaultKsMinDraws[2] = {2048, 2048};
constexpr uint64_t kKsLongDraws = 4096;
constexpr uint64_t kKsLongRounds = 4;   // 1-wave workgroups: 8 GiB launches (4 rounds) 6755 -> 6986 GB/s at 4096
constexpr uint64_t kKsMinSpan = 256;          // fewest draws per lane for small launches
// DG1 with a zero prefix (compress > 1): 512 draws per lane by default, so the
// waves that skip the PRNG cover more of each block's prefix (d1 c2: 6413 ->
// 6694 GB/s; at c1 the extra jumps cost: 5896 -> 5347, profiles/r02/diag/k2_xcd.log)
constexpr uint64_t kDgenPrefixMinDraws = 512;
// measured on MI355X (tools/k2_lab.py, profiles/r02/diag/k2_lab_r2e.log):
// 512-B row pieces, 4-wave workgroups, 1024 draws per lane and sc1 stores for
// both modes (K2 6010 vs 5803 GB/s at 2048 draws; DG1 c1 5933 / c2 6158 vs
// 5187 / 5409 for the round-1 DG1 shape of 128-B pieces and 2 waves).  With
// 1024 draws per lane a 1 MiB DG1 block is 128 lanes, so whole waves fall
// inside a zero prefix and skip the PRNG.
// XCD groups (k_keystream remaps workgroups so each XCD writes runs of
// adjacent waves' lane regions instead of every 8th workgroup) and 1-wave
// workgroups (a finished wave frees its slot without waiting for three
// others).  One process, interleaved (profiles/r02/diag/ks/ks_xcd_sweep.log):
//   K2 80 GiB, 4096 draws:   4 waves, dealing order 6475 -> 1 wave, groups of 16: 6737 GB/s
//   K2 8 GiB, 2048 draws:    6551 -> 7007
//   DG1 c1 80 GiB / 8 GiB:   6409 / 6561 -> 6646 / 6774
//   DG1 c2 (zero prefix, 512 draws): 6061 -> 6682 with 4 waves, groups of 32
//                            (1 wave, groups of 16: 6251)
constexpr int kDefaultKsXcdWaves = 16;
constexpr KsShape kDefaultKsShape[2] = {{64, 1, 0, kStoreSC1, kDefaultKsXcdWaves},
                                        {64, 1, 0, kStoreSC1, kDefaultKsXcdWaves}};
constexpr int kDgenPrefixWaves = 4, kDgenPrefixXcdWaves = 32;
// DG1 with a zero prefix, from this many whole 1 MiB blocks per launch: the
// prefixes as whole 4 KiB granules in the fill's store shape (k_zero_prefix),
// then the keystream over the tails alone (s3dg_set_dgen_zero_split;
// DESIGN.md §5.3).  The zero launch's occupancy cap and store policy.
// The zero launch's shape per prefix class, measured (tools/dg1_split_lab.py,
// profiles/r05/i, j: ten 8 GiB DG1 objects, one launch each / all in one):
// prefixes that end on a 64-B line (c = 2, 4, ...): 4-wave workgroups, 5
// resident per CU, nt sc1 stores, after the tails' launch on the same stream
// (c2 0.843 / 0.854, c4 0.875 against one keystream launch's 0.781 / 0.848,
// 0.842); mid-line prefixes (c = 3, 1.5, ...): 1-wave workgroups, 14 per CU,
// nt sc1, on a side stream concurrent with the tails (c3 0.794 / 0.866, c1.5
// 0.857 against 0.735 / 0.779, 0.729).  Index: [0] line-aligned, [1] mid-line.
constexpr uint64_t kDefaultDgenZeroSplit = 64;
constexpr int kZeroPrefixWaves[2] = {4, 1}, kZeroPrefixOcc[2] = {5, 14};
constexpr int kZeroPrefixStore[2] = {kStoreNTSC1, kStoreNTSC1}, kZeroPrefixOverlap[2] = {0, 1};

// Launch state private to one stream: the tile-record map of tiled launches
// and the batch-descriptor staging.  Launches on one stream are ordered by
// the stream, so a launch may rewrite the map as soon as it is enqueued after
// the previous one; launches on different streams share nothing and never
// wait on each other.
struct StreamState {
    std::mutex mu;                     // one enqueuing thread per stream at a time
    TileRec *tiles = nullptr;          // records of uniform tiled launches (device), grown on demand
    uint64_t tile_cap = 0;
    // batch records: two maps, so sub-batch k+1's k_batch_map (on `up`) runs
    // while sub-batch k's fill (on the stream) reads the other one
    TileRec *btiles[2] = {nullptr, nullptr};
    uint64_t btile_cap[2] = {0, 0};
    hipEvent_t mapped[2] = {nullptr, nullptr};   // map [i] written (on up)
    hipEvent_t filled[2] = {nullptr, nullptr};   // fill reading map [i] done (on the stream)
    int bnext = 0;
    hipStream_t up = nullptr;          // batch entry uploads + record maps (overlap the previous fill)
    // DG1 zero-prefix launches concurrent with their tails (s3dg_set_dgen_zero_split overlap)
    hipStream_t zs = nullptr;
    hipEvent_t zfork = nullptr, zjoin = nullptr;
    struct Stage {
        s3dg_obj_desc *host = nullptr, *dev = nullptr;   // pinned staging / device copy
        uint64_t *rec_lo = nullptr;    // device: record offset of each object (tile layouts)
        void *scan_tmp = nullptr;      // device: scan scratch
        size_t scan_tmp_bytes = 0;
        uint64_t cap = 0;
        hipEvent_t uploaded = nullptr;  // host staging may be rewritten
        hipEvent_t consumed = nullptr;  // device copy may be freed (k_batch_map done; both on `up`)
    } stage[2];
    int next = 0;
    // queue counters of persistent keystream launches on this stream
    KsCounters ks;
    // lifetime (under the context's mu): users holding the state, and whether
    // s3dg_stream_release has taken it out of the context's map; the last
    // holder of a released state drains the stream and frees it
    int refs = 0;
    bool dead = false;
};

struct s3dg_ctx {
    int device = 0;
    int cus = 256;                     // compute units (sizes small keystream launches)
    // store cache policy: sc1 (write, then drop the line from
    // L2) for batches, nt sc1 for streams, measured best
    int store_stream = kDefaultStoreStream, store_batch = kDefaultStoreBatch;
    int store_dense = kDefaultStoreDense;   // batch launches in the dense layout
    int waves_per_block = 0;           // 0 = auto: 2 for streams, 1 for batches (measured)
    // resident fill workgroups per CU (0 = hardware max); measured on MI355X
    // (DESIGN.md §5.1): 14 for 2-wave stream blocks, no cap for 1-wave batch blocks
    int occ_stream = kDefaultOccStream, occ_batch = kDefaultOccBatch;
    int batch_rt_floor = kDefaultBatchRtFloor;   // batch kernel's wall-clock store floor (ticks; -1 = per launch)
    uint32_t prefetch_tiles = kDefaultPrefetch;   // batch tile-record prefetch distance
    uint32_t tile_shift = 0;           // batch tile = 2^tile_shift blocks; 0 = per launch
    bool tile_force_dense = false;     // batch: one record per 4 KiB granule when the layout allows
    // batch: objects of fewer blocks go to a launch of their own with their own
    // tile size (0 = one launch per sub-batch)
    uint32_t split_blocks = kDefaultSplitBlocks;
    // k_keystream launch shapes, [0] npz keystream, [1] DG1
    KsShape ks[2] = {kDefaultKsShape[0], kDefaultKsShape[1]};
    uint64_t ks_min_draws[2] = {kDefaultKsMinDraws[0], kDefaultKsMinDraws[1]};   // draws per lane
    bool ks_auto_waves[2] = {true, true}, ks_auto_xcd[2] = {true, true};          // not set by the caller
    int ks_persist = -1;               // persistent keystream launches from this many rounds (-1: default)
    uint64_t dgen_zero_split = kDefaultDgenZeroSplit;   // DG1 zero prefix + tail launches from this many blocks
    int zp_waves = -1, zp_occ = -1, zp_store = -1, zp_overlap = -1;   // -1: per prefix class (kZeroPrefix*)
    int64_t ks_tail = -1;              // one-object DG1 launches: chunks in half-length lanes at the end (-1: auto)
    void *base_dev = nullptr;          // 4 KiB base block in HBM
    uint8_t base_host[kBlk];
    // tile maps and batch staging, one set per stream (s3dg::StreamState)
    std::map<hipStream_t, StreamState *> streams;
    int stream_tiles = kDefaultStreamTiles;   // uniform streams through the tiled batch kernel
    std::map<std::pair<uint64_t, uint64_t>, uint64_t *> jtabs;   // (lpc << 32 | span, z0) -> device jump table
    void *crc_tab = nullptr;           // slicing-by-8 tables (device)
    uint32_t *crc_seg = nullptr;       // per-segment CRCs (device)
    uint64_t crc_seg_cap = 0;
    std::mutex crc_mu;
    ZcTuner tune[3];                   // per zero class (under mu)
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

// Zero-prefix class of compress (f_num, f_den): kZcLines when const_len =
// 4096 f_num / f_den is a multiple of 64 (64 f_num / f_den whole), i.e. the
// prefix ends on a 64-B line in every block; kZcMidHeavy when it ends inside
// a line and covers at least half the block; kZcNone otherwise.
static inline int zero_class(uint64_t f_num, uint64_t f_den) {
    if (f_num == 0 || f_den == 0) return kZcNone;
    if ((f_num * 64) % f_den == 0) return kZcLines;
    return 2 * f_num >= f_den ? kZcMidHeavy : kZcNone;
}

// zclass: the launch's zero-prefix class (zero_class; batches: the class of
// most of its blocks); picks the batch kernel's occupancy cap and store floor
// when they are not set explicitly (s3dg_set_occupancy, s3dg_set_batch_pace).
LaunchCfg cfg_for(s3dg_ctx *c, bool batch = false, int zclass = kZcNone) {
    LaunchCfg lc;
    lc.store = batch ? c->store_batch : c->store_stream;
    lc.waves_per_block = c->waves_per_block ? c->waves_per_block : (batch ? 1 : 2);
    const int occ = !batch ? c->occ_stream : c->occ_batch >= 0 ? c->occ_batch
                                           : zclass == kZcLines ? kOccZeroLines : 0;
    lc.dyn_lds = occupancy_lds(occ, kFillStaticLds);
    if (batch)
        lc.rt_floor = c->batch_rt_floor >= 0 ? (uint32_t)c->batch_rt_floor
                                             : zclass == kZcMidHeavy ? kRtFloorMidZeros : 0u;
    lc.prefetch_tiles = batch ? c->prefetch_tiles : 0;
    return lc;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

bool tune_enabled() {
    static const bool on = [] {
        const char *e = getenv("S3DG_ZC_TUNE");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Mean rate (GB/s) of candidate q's last kTuneKeep timed launches (0: none).
double tune_mean(const ZcTuner &T, int q) {
    const int n = std::min(T.samples[q], kTuneKeep);
    if (n == 0) return 0.0;
    double sum = 0.0;
    for (int k = 0; k < n; ++k) sum += T.recent[q][k];
    return sum / n;
}

// A launch of class zc writing `bytes`: the candidate to run (0 = the fitted
// rule, 1 = plain) and whether to time it (*timed, events in *probe).
int tune_pick(s3dg_ctx *c, int zc, uint64_t bytes, bool *timed, ZcTuner::Pending *probe) {
    *timed = false;
    if (zc != kZcMidHeavy || c->occ_batch >= 0 || c->batch_rt_floor >= 0 || !tune_enabled()) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    ZcTuner &T = c->tune[zc];
    // harvest finished measurements (never waits)
    int probed = 0;   // new samples of the candidate not chosen
    for (size_t k = 0; k < T.pend.size();) {
        ZcTuner::Pending &p = T.pend[k];
        if (hipEventQuery(p.b) != hipSuccess) {
            (void)hipGetLastError();
            ++k;
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess && ms > 0.f) {
            if (!T.warm) {
                T.warm = true;   // the context's first timed launch: warm-up, not a sample
            } else {
                T.recent[p.cand][T.samples[p.cand] % kTuneKeep] = p.bytes / (ms * 1e6);
                ++T.samples[p.cand];
                if (p.cand != T.best) ++probed;
            }
        }
        (void)hipGetLastError();
        T.spare.push_back(p.a);
        T.spare.push_back(p.b);
        T.pend[k] = T.pend.back();
        T.pend.pop_back();
    }
    if (T.samples[0] >= kTuneFirst && T.samples[1] >= kTuneFirst) {
        const double mean[2] = {tune_mean(T, 0), tune_mean(T, 1)};
        // switch only when the other candidate is clearly faster (hysteresis)
        if (mean[1 - T.best] > mean[T.best] * (1.0 + kTuneMargin)) {
            T.best = 1 - T.best;
            T.interval = kTuneReprobe;
        } else if (probed) {   // a probe confirmed the choice: probe less often
            T.interval = std::min(2 * T.interval, kTuneReprobeMax);
        }
    }
    if (bytes < kTuneMinBytes) return T.best;
    int cand;
    if (T.issued[0] < (uint64_t)kTuneFirst + 1 || T.issued[1] < (uint64_t)kTuneFirst) {
        cand = (int)(T.launches & 1);   // rule, plain, rule, plain (the first launch is the warm-up)
    } else {
        if (T.next_probe == 0) T.next_probe = T.launches + T.interval;
        cand = T.best;
        if (T.launches >= T.next_probe) {
            cand = 1 - T.best;
            T.next_probe = T.launches + T.interval;
        }
    }
    if (T.pend.size() < 16) {
        for (int q = 0; q < 2; ++q) {
            hipEvent_t &e = q ? probe->b : probe->a;
            if (!T.spare.empty()) {
                e = T.spare.back();
                T.spare.pop_back();
            } else if (hipEventCreate(&e) != hipSuccess) {
                (void)hipGetLastError();
                if (q) T.spare.push_back(probe->a);
                return cand;
            }
        }
        probe->bytes = (double)bytes;
        probe->cand = cand;
        *timed = true;
    }
    ++T.launches;
    ++T.issued[cand];
    return cand;
}

// Record the timed launch's events around it (start before, end after).  A
// probe whose launch failed (launched = false at the end mark) records no rate:
// its events go straight back to the spares (its near-zero elapsed
// time would otherwise enter the medians as a huge GB/s sample).
void tune_mark(s3dg_ctx *c, int zc, const ZcTuner::Pending &probe, bool end, hipStream_t s, bool launched = true) {
    if (end && !launched) {
        std::lock_guard<std::mutex> g(c->mu);
        c->tune[zc].spare.push_back(probe.a);
        c->tune[zc].spare.push_back(probe.b);
        return;
    }
    (void)hipEventRecord(end ? probe.b : probe.a, s);
    if (end) {
        std::lock_guard<std::mutex> g(c->mu);
        c->tune[zc].pend.push_back(probe);
    }
}

// Batch tile size: every object's last tile is ragged, and its blocks past
// the object's end are workgroups that start, load the record and exit.
// Smaller tiles cut those, at one 64-B record (and one more record miss per
// XCD) per tile.  Pick the tile size that minimises launched workgroups +
// kTileCost x records.
constexpr uint64_t kTileCost = 2;

uint32_t pick_tile_shift(const uint64_t (&ntiles)[kTileShiftMax + 1]) {
    uint32_t best = kTileShiftMax;
    uint64_t best_cost = UINT64_MAX;
    for (uint32_t sh = kTileShiftMax; sh >= kTileShiftAutoMin; --sh) {
        const uint64_t cost = (ntiles[sh] << sh) + kTileCost * ntiles[sh];
        if (cost < best_cost) { best_cost = cost; best = sh; }
    }
    return best;
}

}  // namespace

namespace s3dg {

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

PrefixParams random_layout_prefix() {
    PrefixParams pp{};
    pp.unique = 0xFFFFFFFFu;            // block i seeded entropy + i
    pp.f_den = 0;                       // generate_random_data layout
    pp.m_unique = fastmod_magic(1);
    pp.m_fden = fastmod_magic(1);
    return pp;
}

LaunchCfg ctx_stream_cfg(const s3dg_ctx *c) { return cfg_for(const_cast<s3dg_ctx *>(c)); }
const void *ctx_base(const s3dg_ctx *c) { return c->base_dev; }

}  // namespace s3dg

extern "C" {

const char *s3dg_last_error(void) { return g_err.c_str(); }
const char *s3dg_version(void) { return "s3dlio_amd 0.1.0 (gfx950)"; }

// The source digest this library was built from (build.py compiles it in;
// the marker lets build.py read it from the file without loading it).
#ifndef S3DG_BUILD_DIGEST
#define S3DG_BUILD_DIGEST "unknown-digest00"
#endif
static const char kBuildDigestRecord[] __attribute__((used)) = "S3DG_BUILD_DIGEST=" S3DG_BUILD_DIGEST;
const char *s3dg_build_digest(void) { return kBuildDigestRecord + sizeof("S3DG_BUILD_DIGEST=") - 1; }

uint64_t s3dg_unique_blocks(uint64_t nblocks, uint64_t dedup) {
    const uint64_t d = dedup == 0 ? 1 : dedup;
    if (d <= 1) return nblocks;
    double r = std::round((double)nblocks / (double)d);   // f64::round, half away
    if (r < 1.0) r = 1.0;
    return (uint64_t)r;
}

int s3dg_zero_class(uint32_t f_num, uint32_t f_den) { return zero_class(f_num, f_den); }

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
    base_from_seed(kDefaultBaseSeed, c->base_host);
    e = hipMemcpy(c->base_dev, c->base_host, kBlk, hipMemcpyHostToDevice);
    if (e != hipSuccess) { s3dg_ctx_destroy(c); return hipfail(e, "hipMemcpy(base block)"); }
    *out = c;
    return S3DG_OK;
}

// Frees one stream's launch state; the caller has drained the stream (and
// its upload stream).
static void stream_state_free(StreamState *S) {
    if (S->tiles) (void)hipFree(S->tiles);
    for (int q = 0; q < 2; ++q) {
        if (S->btiles[q]) (void)hipFree(S->btiles[q]);
        if (S->mapped[q]) (void)hipEventDestroy(S->mapped[q]);
        if (S->filled[q]) (void)hipEventDestroy(S->filled[q]);
    }
    for (auto &G : S->stage) {
        if (G.host) (void)hipHostFree(G.host);
        for (void *p : {(void *)G.dev, (void *)G.rec_lo, G.scan_tmp})
            if (p) (void)hipFree(p);
        if (G.uploaded) (void)hipEventDestroy(G.uploaded);
        if (G.consumed) (void)hipEventDestroy(G.consumed);
    }
    if (S->up) (void)hipStreamDestroy(S->up);
    if (S->zs) (void)hipStreamDestroy(S->zs);
    for (hipEvent_t e : {S->zfork, S->zjoin})
        if (e) (void)hipEventDestroy(e);
    if (S->ks.dev) (void)hipFree(S->ks.dev);
    delete S;
}

int s3dg_ctx_destroy(s3dg_ctx *c) {
    if (!c) return S3DG_OK;
    DeviceScope ds(c->device);
    (void)hipDeviceSynchronize();
    if (c->base_dev) (void)hipFree(c->base_dev);
    for (auto &kv : c->streams) stream_state_free(kv.second);
    for (auto &kv : c->jtabs) (void)hipFree(kv.second);
    if (c->crc_tab) (void)hipFree(c->crc_tab);
    if (c->crc_seg) (void)hipFree(c->crc_seg);
    for (auto &T : c->tune) {
        for (auto &p : T.pend) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : T.spare) (void)hipEventDestroy(e);
    }
    delete c;
    return S3DG_OK;
}

// a context keeps tile maps and batch staging per stream it has
// seen; a caller that retires a stream releases them here (after draining
// the stream), so short-lived streams do not accumulate device memory and a
// reused handle value starts from fresh state.
int s3dg_stream_release(s3dg_ctx *c, void *stream) {
    CTX_SCOPE(c);
    StreamState *S = nullptr;
    {
        std::lock_guard<std::mutex> g(c->mu);
        auto it = c->streams.find((hipStream_t)stream);
        if (it == c->streams.end()) return S3DG_OK;
        S = it->second;
        c->streams.erase(it);
        S->dead = true;
        ++S->refs;                               // held by this release until the drain below
    }
    hipError_t e;
    {
        std::lock_guard<std::mutex> g(S->mu);    // wait for an enqueue in progress
        e = hipStreamSynchronize((hipStream_t)stream);
        if (e == hipSuccess && S->up) e = hipStreamSynchronize(S->up);
        if (e == hipSuccess && S->zs) e = hipStreamSynchronize(S->zs);
    }
    bool last;
    {
        std::lock_guard<std::mutex> g(c->mu);
        last = --S->refs == 0;
    }
    if (last) stream_state_free(S);              // else the last holder drains and frees it (StreamLock)
    HIP_TRY(e, "hipStreamSynchronize(release)");
    return S3DG_OK;
}

// Streams with launch state in this context (diagnostics and tests).
int s3dg_stream_state_count(s3dg_ctx *c, uint64_t *n) {
    if (!c || !n) return fail(S3DG_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(c->mu);
    *n = c->streams.size();
    return S3DG_OK;
}

int s3dg_ctx_device(s3dg_ctx *c, int *device) {
    if (!c || !device) return fail(S3DG_EINVAL, "null argument");
    *device = c->device;
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
    c->store_dense = on ? kStoreNT : kDefaultStoreDense;
    return S3DG_OK;
}

int s3dg_set_store_policy(s3dg_ctx *c, int stream_policy, int batch_policy) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (stream_policy > kStoreNTSC1 || batch_policy > kStoreNTSC1)
        return fail(S3DG_EINVAL, "store policy must be 0 (plain), 1 (nt), 2 (sc1), 3 (nt sc1) or negative (default)");
    c->store_stream = stream_policy < 0 ? kDefaultStoreStream : stream_policy;
    c->store_batch = batch_policy < 0 ? kDefaultStoreBatch : batch_policy;
    c->store_dense = batch_policy < 0 ? kDefaultStoreDense : batch_policy;
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

int s3dg_set_batch_pace(s3dg_ctx *c, int ticks) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (ticks > 100000) return fail(S3DG_EINVAL, "store floor must be at most 100000 ticks (1 ms)");
    c->batch_rt_floor = ticks < 0 ? kDefaultBatchRtFloor : ticks;
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
    if (blocks > 1) {
        while ((1u << sh) < blocks) ++sh;
        if ((1u << sh) != blocks || sh < kTileShiftMin || sh > kTileShiftMax)
            return fail(S3DG_EINVAL, "tile blocks must be 0 (per launch), 1 (dense), 2, 4, 8, 16, 32 or 64");
    }
    c->tile_shift = sh;
    c->tile_force_dense = blocks == 1;
    return S3DG_OK;
}

int s3dg_query_zero_tune(s3dg_ctx *c, int zclass, int *best, double *rule_gbs, double *plain_gbs, uint64_t *timed) {
    if (!c || zclass < 0 || zclass > 2) return fail(S3DG_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(c->mu);
    const ZcTuner &T = c->tune[zclass];
    if (best) *best = T.best;
    if (rule_gbs) *rule_gbs = tune_mean(T, 0);
    if (plain_gbs) *plain_gbs = tune_mean(T, 1);
    if (timed) *timed = T.launches;
    return S3DG_OK;
}

int s3dg_set_batch_split(s3dg_ctx *c, int blocks) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    c->split_blocks = blocks < 0 ? kDefaultSplitBlocks : (uint32_t)blocks;
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
    c->ks_auto_waves[mode] = waves == 0;
    c->ks[mode].wgs_per_cu = wgs_per_cu;
    c->ks[mode].store = store_policy < 0 ? def.store : store_policy;
    c->ks_min_draws[mode] = min_lane_draws ? min_lane_draws : kDefaultKsMinDraws[mode];
    return S3DG_OK;
}

int s3dg_set_keystream_xcd_group(s3dg_ctx *c, int mode, uint32_t waves) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (mode != 0 && mode != 1) return fail(S3DG_EINVAL, "mode must be 0 (keystream) or 1 (dgen)");
    if (waves > 4096 || (waves & (waves - 1))) return fail(S3DG_EINVAL, "waves per XCD group must be 0 or a power of two <= 4096");
    std::lock_guard<std::mutex> g(c->mu);
    c->ks[mode].xcd_waves = waves ? (int)waves : kDefaultKsXcdWaves;
    c->ks_auto_xcd[mode] = waves == 0;
    return S3DG_OK;
}

int s3dg_set_keystream_persist(s3dg_ctx *c, int rounds) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    c->ks_persist = rounds < 0 ? -1 : rounds;
    return S3DG_OK;
}

int s3dg_set_dgen_zero_split(s3dg_ctx *c, int chunks, int waves, int occupancy, int store, int overlap) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    if (waves != 0 && waves != 1 && waves != 2 && waves != 4 && waves >= 0)
        return fail(S3DG_EINVAL, "waves must be 1, 2 or 4 (0 or negative: default)");
    if (occupancy > 64) return fail(S3DG_EINVAL, "occupancy must be <= 64 workgroups per CU");
    if (store > kStoreNTSC1) return fail(S3DG_EINVAL, "store policy must be 0, 1, 2, 3 or negative");
    std::lock_guard<std::mutex> g(c->mu);
    c->dgen_zero_split = chunks < 0 ? kDefaultDgenZeroSplit : (uint64_t)chunks;
    c->zp_waves = waves <= 0 ? -1 : waves;
    c->zp_occ = occupancy < 0 ? -1 : occupancy;
    c->zp_store = store < 0 ? -1 : store;
    c->zp_overlap = overlap < 0 ? -1 : (overlap ? 1 : 0);
    return S3DG_OK;
}

int s3dg_set_keystream_tail(s3dg_ctx *c, int chunks) {
    if (!c) return fail(S3DG_EINVAL, "null context");
    std::lock_guard<std::mutex> g(c->mu);
    c->ks_tail = chunks < 0 ? -1 : chunks;
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
    HIP_TRY(fill_occupancy(cfg_for(c, batch != 0, batch == 2 ? kZcLines : kZcNone), batch != 0, wgs_per_cu),
            "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    return S3DG_OK;
}

// The stream's launch state (created on first use), held and locked for the
// scope: one enqueuing thread per stream at a time, and a concurrent
// s3dg_stream_release never frees a state someone still holds (ADVICE r03:
// the holder that drops the last reference of a released state drains the
// stream and frees it).
class StreamLock {
public:
    StreamLock(s3dg_ctx *c, hipStream_t s) : c_(c), s_(s) {
        {
            std::lock_guard<std::mutex> g(c->mu);
            StreamState *&S = c->streams[s];
            if (!S) S = new StreamState();
            S_ = S;
            ++S_->refs;
        }
        S_->mu.lock();
    }
    ~StreamLock() {
        S_->mu.unlock();
        bool last;
        {
            std::lock_guard<std::mutex> g(c_->mu);
            last = --S_->refs == 0 && S_->dead;
        }
        if (last) {
            (void)hipStreamSynchronize(s_);
            if (S_->up) (void)hipStreamSynchronize(S_->up);
            if (S_->zs) (void)hipStreamSynchronize(S_->zs);
            stream_state_free(S_);
        }
    }
    StreamState *get() const { return S_; }
    StreamLock(const StreamLock &) = delete;
    StreamLock &operator=(const StreamLock &) = delete;

private:
    s3dg_ctx *c_;
    hipStream_t s_;
    StreamState *S_ = nullptr;
};

// At least `tiles` records in the stream's map.  Earlier launches on this
// stream may still read the old map: growing drains the stream first.
// Caller holds S->mu.
static int tiles_reserve(StreamState *S, uint64_t tiles, hipStream_t s) {
    if (tiles <= S->tile_cap) return S3DG_OK;
    HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize(tile map)");
    if (S->tiles) (void)hipFree(S->tiles);
    S->tiles = nullptr;
    S->tile_cap = 0;
    const uint64_t cap = tiles < 4096 ? 4096 : tiles + tiles / 4;
    HIP_TRY(hipMalloc(&S->tiles, cap * sizeof(TileRec)), "hipMalloc(tile map)");
    S->tile_cap = cap;
    return S3DG_OK;
}

// n_objs objects of obj_size bytes at dst + j*stride, entropy seed_base +
// ((first_obj + j) << 32), prefix parameters pp.  Large streams whose objects
// all start on the same 4 KiB granule (mod 8) run through the tiled batch
// kernel; the rest through the 2D stream kernel.
// held: the stream's state when the caller already holds it (batch sub-batches).
static int fill_uniform(s3dg_ctx *c, uint8_t *dst, uint64_t obj_size, uint64_t stride, uint64_t n_objs,
                        const PrefixParams &pp, uint64_t seed_base, uint64_t first_obj, hipStream_t s,
                        StreamState *held = nullptr) {
    const uint64_t nb = (obj_size + kBlk - 1) / kBlk;
    const uint32_t lead = (uint32_t)(((uintptr_t)dst >> 12) & 7);
    if (c->stream_tiles && (n_objs == 1 || stride % (8 * kBlk) == 0) && n_objs * nb >= kStreamTilesMinBlocks &&
        nb + lead < (1ull << 31)) {
        uint64_t ntiles[kTileShiftMax + 1] = {};
        for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh)
            ntiles[sh] = n_objs * ((nb + lead + (1ull << sh) - 1) >> sh);
        const uint32_t tshift = c->tile_shift ? c->tile_shift : pick_tile_shift(ntiles);
        const uint64_t tpo = (nb + lead + (1ull << tshift) - 1) >> tshift;
        std::unique_ptr<StreamLock> SL;
        if (!held) SL.reset(new StreamLock(c, s));
        StreamState *S = held ? held : SL->get();
        if (int r = tiles_reserve(S, n_objs * tpo, s)) return r;
        // the prefix's class from its exact length (pp: 4096 f_num / f_den = floor_len + rem / f_den)
        const int zc = pp.f_den == 0 || (pp.floor_len == 0 && pp.rem == 0) ? kZcNone
                       : pp.rem == 0 && (pp.floor_len & 63u) == 0      ? kZcLines
                       : 2 * (uint64_t)pp.floor_len >= kBlk            ? kZcMidHeavy
                                                                        : kZcNone;
        bool timed = false;
        ZcTuner::Pending probe{};
        const int cand = tune_pick(c, zc, obj_size * n_objs, &timed, &probe);
        if (timed) tune_mark(c, zc, probe, false, s);
        LaunchCfg lc = cfg_for(c, true, cand ? kZcNone : zc);
        if (zc == kZcNone && c->batch_rt_floor < 0 && nb >= kRtFloorLargeBlocks) lc.rt_floor = kRtFloorLargeUniform;
        const hipError_t le = launch_fill_uniform_tiles(lc, dst, obj_size, stride, n_objs, (uint32_t)tpo, tshift, lead,
                                                        seed_base + (first_obj << 32), pp, S->tiles, c->base_dev, s);
        if (timed) tune_mark(c, zc, probe, true, s, le == hipSuccess);
        HIP_TRY(le,
                "launch k_fill_batch(stream)");
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
    const PrefixParams pp = random_layout_prefix();
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
        pp = random_layout_prefix();
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

// Mixed-size batch ("Batches"): the descriptors are cut into
// sub-batches (16 Ki objects first, doubling to 256 Ki) so the host's pass
// over sub-batch k+1 overlaps the GPU's fill of sub-batch k.  Per sub-batch
// the host makes one pass on up to 8 threads: it validates, counts slots and
// copies the 40-B descriptors into pinned staging (empty ones squeezed out
// afterwards); the upload runs on the stream's side
// stream, where a device scan of the tile counts gives each object's record
// offset and k_batch_map derives prefix parameters and tile records.
// Record layout per sub-batch (cost model below):
//   * tiles of 2^tshift blocks (2..64) per object, the object's block 0 at
//     slot `lead` = its 4 KiB granule (mod 8): XCD-aligned, dead slots at
//     both ends of every object;
//   * dense (tshift 0): objects 4 KiB-aligned, sorted and non-overlapping;
//     one record per 4 KiB granule of the sub-batch's address range, so slot
//     = granule and only gaps are dead.
// Descriptors are checked per sub-batch: on an error the objects of earlier
// sub-batches may already be enqueued.
constexpr uint64_t kBatchSubFirst = 16384, kBatchSubMax = 262144;
// relative costs in units of one live 4 KiB block, fitted
// to forced dense / 8-block layouts of uniform 7..26-block objects with the
// dense launches' nt sc1 stores (profiles/r02/diag/batch_lab_store_cost.log)
constexpr double kDeadSlotCost = 0.4, kRecordCost = 0.05;
// Among tile sizes, the costs measured on config 4's mixed sizes (forced 64 /
// 32 / 16 / 8-block tiles: 7249 / 7215 / 7152 / 6991 GB/s, one process,
// profiles/r03/diag/cfg4/cfg4_tiles.log) fit a dead slot at ~0 and a record at
// ~0.25 live blocks: a tile's dead slots find its record already in the
// scalar cache, while each extra record is one more miss on a workgroup's
// critical path.  The first model (above) picked 16-block tiles there; it
// still decides dense vs tiled, as fitted.
constexpr double kDeadSlotCostTiled = 0.1, kRecordCostTiled = 0.25;
constexpr int kPrepParts = 8;                   // host threads per sub-batch pass
constexpr uint64_t kPrepMinPerPart = 8192;      // descriptors below which a pass stays single-threaded

// A few persistent host threads for the batch passes: run(parts, fn) calls
// fn(0..parts-1), part 0 in the caller.  One run at a time; a second caller
// meanwhile runs its parts itself.
class PrepPool {
public:
    static PrepPool &get() {
        static PrepPool *p = new PrepPool();   // never destroyed: workers outlive main
        return *p;
    }
    void run(int parts, const std::function<void(int)> &fn) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock() || parts <= 1) {
            for (int q = 0; q < parts; ++q) fn(q);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            parts_ = parts;
            next_.store(1);
            left_ = parts - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        for (int q; (q = next_.fetch_add(1)) < parts;) finish_one(q);
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return left_ == 0; });
        fn_ = nullptr;
    }

private:
    PrepPool() {
        for (int k = 0; k < kPrepParts - 1; ++k) std::thread([this] { loop(); }).detach();
    }
    void finish_one(int q) {
        (*fn_)(q);
        std::lock_guard<std::mutex> g(mu_);
        if (--left_ == 0) done_cv_.notify_all();
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
            }
            for (int q; (q = next_.fetch_add(1)) < parts_;) finish_one(q);
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)> *fn_ = nullptr;
    int parts_ = 0, left_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
};

// Pass 1 over descriptors [k0, k1): validation, slot counts per tile size,
// dense-layout test.
struct BatchScan {
    uint64_t m = 0, blocks = 0, zc_blocks[3] = {}, ntiles[kTileShiftMax + 1] = {};
    // objects below the split threshold: count, blocks, tiles per tile size
    uint64_t ms = 0, blocks_s = 0, ntiles_s[kTileShiftMax + 1] = {};
    uint64_t first_off = 0, last_end = 0;
    bool dense_ok = true;
    // uniform: every non-empty object has the first's size, dedup and ratio,
    // at a constant stride (>= size) with entropy stepping by 2^32, i.e. the
    // batch is a stream (s3dg_fill_controlled_stream's layout and seeds)
    bool uni = true;
    s3dg_obj_desc ufirst{}, ulast{};
    uint64_t ustride = 0;
    int err = S3DG_OK;
    const char *msg = nullptr;
};

// Does object b continue the uniform run whose last object is a (stride 0: not yet known)?
static inline bool uni_next(const s3dg_obj_desc &first, const s3dg_obj_desc &a, const s3dg_obj_desc &b,
                           uint64_t &stride) {
    if (b.size != first.size || b.dedup != first.dedup || b.f_num != first.f_num || b.f_den != first.f_den ||
        b.entropy - a.entropy != (1ull << 32) || b.dst_off < a.dst_off)
        return false;
    const uint64_t st = b.dst_off - a.dst_off;
    if (stride == 0) stride = st;
    return st == stride && st >= first.size;
}

static void batch_scan(const s3dg_obj_desc *__restrict d, uint64_t k0, uint64_t k1, uintptr_t base, BatchScan &P,
                       s3dg_obj_desc *__restrict out, uint64_t split) {
    // accumulators in registers (P aliases nothing, but the compiler cannot
    // know that across the staging stores); the checks fold into one flag
    uint64_t m = 0, blocks = 0, zc_blocks[3] = {}, first = 0, last = 0, nt[kTileShiftMax + 1] = {};
    uint64_t ms = 0, blocks_s = 0, nts[kTileShiftMax + 1] = {};
    bool dense = true, bad = false, uni = true;
    uint32_t zc_num = 0, zc_den = 1;   // last compress seen and its zero_class
    int zc = kZcNone;
    s3dg_obj_desc ufirst{}, uprev{};
    uint64_t ustride = 0;
    for (uint64_t k = k0; k < k1; ++k) {
        const s3dg_obj_desc o = d[k];
        out[k - k0] = o;   // staged as is; empty objects are squeezed out afterwards (rare)
        if (o.size == 0) continue;
        if (m == 0) ufirst = o;
        else uni = uni && uni_next(ufirst, uprev, o, ustride);
        uprev = o;
        const uint64_t nb = (o.size + kBlk - 1) / kBlk;
        bad |= (o.dst_off & 15u) != 0 || o.f_den == 0 || o.f_num >= o.f_den || nb >= (1ull << 31);
        const uint64_t x = nb + (((base + o.dst_off) >> 12) & 7);   // blocks behind the XCD lead
        for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) nt[sh] += (x + (1ull << sh) - 1) >> sh;
        if (nb < split) {
            ++ms;
            blocks_s += nb;
            for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) nts[sh] += (x + (1ull << sh) - 1) >> sh;
        }
        if (m == 0) first = o.dst_off;
        dense = dense && (m == 0 || o.dst_off >= last) && (o.dst_off & (kBlk - 1)) == 0;
        last = o.dst_off + nb * kBlk;
        blocks += nb;
        if (o.f_num != zc_num || o.f_den != zc_den) {
            zc_num = o.f_num;
            zc_den = o.f_den;
            zc = zero_class(o.f_num, o.f_den);
        }
        zc_blocks[zc] += nb;
        ++m;
    }
    if (bad) {   // the first offending descriptor names the error
        for (uint64_t k = k0; k < k1; ++k) {
            const s3dg_obj_desc &o = d[k];
            if (o.size == 0) continue;
            P.err = S3DG_EINVAL;
            if (o.dst_off & 15u) { P.msg = "dst_off must be a multiple of 16"; return; }
            if (o.f_den == 0 || o.f_num >= o.f_den) { P.msg = "need f_num < f_den"; return; }
            if ((o.size + kBlk - 1) / kBlk >= (1ull << 31)) { P.msg = "object larger than 2^31 blocks"; return; }
            P.err = S3DG_OK;
        }
    }
    P.m = m;
    P.blocks = blocks;
    P.ms = ms;
    P.blocks_s = blocks_s;
    for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) P.ntiles_s[sh] = nts[sh];
    for (int k = 0; k < 3; ++k) P.zc_blocks[k] = zc_blocks[k];
    P.first_off = first;
    P.last_end = last;
    P.dense_ok = dense;
    P.uni = uni;
    P.ufirst = ufirst;
    P.ulast = uprev;
    P.ustride = ustride;
    for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) P.ntiles[sh] = nt[sh];
}

int s3dg_fill_controlled_batch(s3dg_ctx *c, void *dst_base, const s3dg_obj_desc *d, uint64_t n,
                               void *stream) {
    CTX_SCOPE(c);
    if (n == 0) return S3DG_OK;
    if (!d) return fail(S3DG_EINVAL, "null descriptor array");
    if (!dst_base || !aligned16(dst_base)) return fail(S3DG_EINVAL, "dst_base must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    const uintptr_t base = (uintptr_t)dst_base;
    StreamLock SL(c, s);
    StreamState *S = SL.get();
    if (!S->up) HIP_TRY(hipStreamCreateWithFlags(&S->up, hipStreamNonBlocking), "hipStreamCreate(upload)");
    for (auto &G : S->stage)
        for (hipEvent_t *ev : {&G.uploaded, &G.consumed})
            if (!*ev) HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming), "hipEventCreate");
    for (int q = 0; q < 2; ++q)
        for (hipEvent_t *ev : {&S->mapped[q], &S->filled[q]})
            if (!*ev) HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming), "hipEventCreate");
    PrepPool &pool = PrepPool::get();
    uint64_t sub = kBatchSubFirst;
    for (uint64_t k0 = 0; k0 < n;) {
        const uint64_t k1 = n - k0 < sub ? n : k0 + sub;
        sub = sub * 2 < kBatchSubMax ? sub * 2 : kBatchSubMax;
        // staging: host buffer free once its last upload finished, device copy
        // once the k_batch_map that read it finished
        StreamState::Stage &G = S->stage[S->next];
        S->next ^= 1;
        HIP_TRY(hipEventSynchronize(G.uploaded), "hipEventSynchronize(batch staging)");
        if (k1 - k0 > G.cap) {
            HIP_TRY(hipEventSynchronize(G.consumed), "hipEventSynchronize(batch staging)");
            if (G.host) (void)hipHostFree(G.host);
            for (void *p : {(void *)G.dev, (void *)G.rec_lo, G.scan_tmp})
                if (p) (void)hipFree(p);
            G.host = nullptr; G.dev = nullptr; G.rec_lo = nullptr; G.scan_tmp = nullptr;
            G.cap = 0; G.scan_tmp_bytes = 0;
            const uint64_t cap = k1 - k0 < 1024 ? 1024 : k1 - k0;
            size_t tmp = 0;
            HIP_TRY(launch_batch_scan(nullptr, cap, kTileShiftMin, 0, nullptr, nullptr, &tmp, S->up),
                    "hipcub scan size");
            HIP_TRY(hipHostMalloc((void **)&G.host, cap * sizeof(s3dg_obj_desc), hipHostMallocDefault),
                    "hipHostMalloc(batch staging)");
            HIP_TRY(hipMalloc((void **)&G.dev, cap * sizeof(s3dg_obj_desc)), "hipMalloc(batch staging)");
            HIP_TRY(hipMalloc((void **)&G.rec_lo, cap * sizeof(uint64_t)), "hipMalloc(batch records)");
            HIP_TRY(hipMalloc(&G.scan_tmp, tmp ? tmp : 1), "hipMalloc(batch scan)");
            G.scan_tmp_bytes = tmp;
            G.cap = cap;
        }
        s3dg_obj_desc *H = G.host;
        // one pass in parts (validate, count, stage), then merged in order
        int parts = (int)((k1 - k0) / kPrepMinPerPart);
        parts = parts < 1 ? 1 : (parts > kPrepParts ? kPrepParts : parts);
        uint64_t cut[kPrepParts + 1];
        for (int q = 0; q <= parts; ++q) cut[q] = k0 + (k1 - k0) * (uint64_t)q / (uint64_t)parts;
        BatchScan part[kPrepParts];
        const uint64_t split = c->split_blocks;
        pool.run(parts, [&](int q) { batch_scan(d, cut[q], cut[q + 1], base, part[q], H + (cut[q] - k0), split); });
        BatchScan P;
        for (int q = 0; q < parts; ++q) {
            const BatchScan &Q = part[q];
            if (Q.err) return fail(Q.err, Q.msg);
            if (Q.m == 0) continue;
            if (P.m == 0) {
                P.first_off = Q.first_off;
                P.ufirst = Q.ufirst;
                P.uni = Q.uni;
                P.ustride = Q.ustride;
            } else {
                if (Q.first_off < P.last_end) P.dense_ok = false;
                // the runs join: Q's first object continues P's last, same stride
                uint64_t st = P.ustride;
                P.uni = P.uni && Q.uni && uni_next(P.ufirst, P.ulast, Q.ufirst, st) &&
                        (Q.ustride == 0 || Q.ustride == st);
                P.ustride = st;
            }
            P.ulast = Q.ulast;
            P.dense_ok = P.dense_ok && Q.dense_ok;
            P.last_end = Q.last_end;
            P.m += Q.m;
            P.blocks += Q.blocks;
            for (int k = 0; k < 3; ++k) P.zc_blocks[k] += Q.zc_blocks[k];
            for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) P.ntiles[sh] += Q.ntiles[sh];
            P.ms += Q.ms;
            P.blocks_s += Q.blocks_s;
            for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) P.ntiles_s[sh] += Q.ntiles_s[sh];
        }
        const uint64_t m = P.m;
        if (m == 0) { k0 = k1; continue; }
        // a uniform sub-batch is a stream: the stream paths (tiled records per
        // 64 blocks, or the 2D kernel with no records at all) instead of a
        // record per tile or granule (config 10's records
        // were 6 % of its traffic).  Unless a batch layout is forced.
        if (P.uni && m >= 2 && !c->tile_shift && !c->tile_force_dense) {
            const uint64_t nb = (P.ufirst.size + kBlk - 1) / kBlk;
            PrefixParams pp;
            if (int r = make_prefix(nb, P.ufirst.dedup, P.ufirst.f_num, P.ufirst.f_den, &pp)) return r;
            if (int r = fill_uniform(c, (uint8_t *)dst_base + P.ufirst.dst_off, P.ufirst.size, P.ustride, m, pp,
                                     P.ufirst.entropy, 0, s, S))
                return r;
            k0 = k1;
            continue;
        }
        const uint64_t lead0 = ((base + P.first_off) >> 12) & 7;
        const uint64_t span = P.dense_ok ? lead0 + (P.last_end - P.first_off) / kBlk : 0;
        // layout: forced (s3dg_set_batch_tile) or least cost
        uint32_t tshift = kTileShiftMax;
        if (c->tile_shift == 0 && c->tile_force_dense && P.dense_ok) tshift = 0;
        else if (c->tile_shift) tshift = c->tile_shift;
        else {
            // tile size by the tiled costs; dense vs the first model's best tiling by the first model
            double best = 1e300, best_t = 1e300;
            for (uint32_t sh = kTileShiftMax; sh >= kTileShiftAutoMin; --sh) {
                const double dead = (double)((P.ntiles[sh] << sh) - P.blocks), recs = (double)P.ntiles[sh];
                const double cost = kDeadSlotCost * dead + kRecordCost * recs;
                const double cost_t = kDeadSlotCostTiled * dead + kRecordCostTiled * recs;
                const bool better = cost < best;
                if (better) best = cost;
#if S3DG_DIAG_OLDTILECOST
                if (better) tshift = sh;   // diagnostic: the first model's tile choice
#else
                (void)better;
                if (cost_t < best_t) { best_t = cost_t; tshift = sh; }
#endif
            }
            if (P.dense_ok && kDeadSlotCost * (double)(span - P.blocks) + kRecordCost * (double)span < best)
                tshift = 0;
        }
        if (m != k1 - k0) {   // squeeze out the empty objects
            uint64_t j = 0;
            for (uint64_t i = 0; i < k1 - k0; ++i)
                if (H[i].size) H[j++] = H[i];
        }
        // two classes (s3dg_set_batch_split): the small objects first, each
        // class with the tile size the tiled cost model picks for it alone
        uint64_t ms = 0;
        uint32_t tsh_s = tshift, tsh_l = tshift;
        if (tshift && !c->tile_shift && split && P.ms > 0 && P.ms < m) {
            uint64_t nt_l[kTileShiftMax + 1] = {};
            for (uint32_t sh = kTileShiftMin; sh <= kTileShiftMax; ++sh) nt_l[sh] = P.ntiles[sh] - P.ntiles_s[sh];
            auto pick = [&](const uint64_t *nt, uint64_t blocks) {
                uint32_t best_sh = kTileShiftMax;
                double best = 1e300;
                for (uint32_t sh = kTileShiftMax; sh >= kTileShiftAutoMin; --sh) {
                    const double cost = kDeadSlotCostTiled * (double)((nt[sh] << sh) - blocks) +
                                        kRecordCostTiled * (double)nt[sh];
                    if (cost < best) { best = cost; best_sh = sh; }
                }
                return best_sh;
            };
            tsh_s = pick(P.ntiles_s, P.blocks_s);
            tsh_l = pick(nt_l, P.blocks - P.blocks_s);
            if (tsh_s != tsh_l) {   // stable partition: small objects first
                ms = P.ms;
                std::vector<s3dg_obj_desc> big;
                big.reserve(m - ms);
                uint64_t j = 0;
                for (uint64_t i = 0; i < m; ++i) {
                    if ((H[i].size + kBlk - 1) / kBlk < split) H[j++] = H[i];
                    else big.push_back(H[i]);
                }
                std::copy(big.begin(), big.end(), H + j);
            }
        }
        const uint64_t recs_s = ms ? P.ntiles_s[tsh_s] : 0;
        const uint64_t recs = tshift == 0 ? span
                              : ms      ? recs_s + (P.ntiles[tsh_l] - P.ntiles_s[tsh_l])
                                        : P.ntiles[tshift];
        const uint64_t rec_alloc = recs;
        // record map tb: free once the fill two sub-batches back has read it
        const int tb = S->bnext;
        S->bnext ^= 1;
        if (rec_alloc > S->btile_cap[tb]) {
            HIP_TRY(hipEventSynchronize(S->filled[tb]), "hipEventSynchronize(tile map)");
            if (S->btiles[tb]) (void)hipFree(S->btiles[tb]);
            S->btiles[tb] = nullptr;
            S->btile_cap[tb] = 0;
            const uint64_t cap = rec_alloc < 4096 ? 4096 : rec_alloc + rec_alloc / 4;
            HIP_TRY(hipMalloc(&S->btiles[tb], cap * sizeof(TileRec)), "hipMalloc(tile map)");
            S->btile_cap[tb] = cap;
        }
        // upload and map on the side stream, overlapping the previous fill
        HIP_TRY(hipMemcpyAsync(G.dev, G.host, m * sizeof(s3dg_obj_desc), hipMemcpyHostToDevice, S->up),
                "hipMemcpyAsync(batch descriptors)");
        HIP_TRY(hipEventRecord(G.uploaded, S->up), "hipEventRecord");
        if (ms) {   // the two classes' scans and records, the small class's records first
            size_t tmp = G.scan_tmp_bytes;
            HIP_TRY(launch_batch_scan(G.dev, ms, tsh_s, base, G.rec_lo, G.scan_tmp, &tmp, S->up), "hipcub scan");
            tmp = G.scan_tmp_bytes;
            HIP_TRY(launch_batch_scan(G.dev + ms, m - ms, tsh_l, base, G.rec_lo + ms, G.scan_tmp, &tmp, S->up),
                    "hipcub scan");
        } else if (tshift) {
            size_t tmp = G.scan_tmp_bytes;
            HIP_TRY(launch_batch_scan(G.dev, m, tshift, base, G.rec_lo, G.scan_tmp, &tmp, S->up), "hipcub scan");
        }
        HIP_TRY(hipStreamWaitEvent(S->up, S->filled[tb], 0), "hipStreamWaitEvent");
        if (ms) {
            HIP_TRY(launch_batch_map(G.dev, ms, G.rec_lo, S->btiles[tb], tsh_s, base, lead0, P.first_off, S->up),
                    "launch k_batch_map");
            HIP_TRY(launch_batch_map(G.dev + ms, m - ms, G.rec_lo + ms, S->btiles[tb] + recs_s, tsh_l, base, lead0,
                                     P.first_off, S->up),
                    "launch k_batch_map");
        } else {
            HIP_TRY(launch_batch_map(G.dev, m, G.rec_lo, S->btiles[tb], tshift, base, lead0, P.first_off, S->up),
                    "launch k_batch_map");
        }
        HIP_TRY(hipEventRecord(G.consumed, S->up), "hipEventRecord");
        HIP_TRY(hipEventRecord(S->mapped[tb], S->up), "hipEventRecord");
        HIP_TRY(hipStreamWaitEvent(s, S->mapped[tb], 0), "hipStreamWaitEvent");
        const int zcls = 2 * P.zc_blocks[kZcLines] > P.blocks      ? kZcLines
                         : 2 * P.zc_blocks[kZcMidHeavy] > P.blocks ? kZcMidHeavy
                                                                   : kZcNone;
        bool timed = false;
        ZcTuner::Pending probe{};
        const int cand = tune_pick(c, zcls, P.blocks * kBlk, &timed, &probe);
        LaunchCfg lcs = cfg_for(c, true, cand ? kZcNone : zcls);
        if (tshift == 0) lcs.store = c->store_dense;
        if (timed) tune_mark(c, zcls, probe, false, s);
        hipError_t le;
        if (ms) {
            le = launch_batch_tiles(lcs, (uint8_t *)dst_base, recs_s, tsh_s, S->btiles[tb], c->base_dev, s);
            if (le == hipSuccess)
                le = launch_batch_tiles(lcs, (uint8_t *)dst_base, recs - recs_s, tsh_l, S->btiles[tb] + recs_s,
                                        c->base_dev, s);
        } else {
            le = launch_batch_tiles(lcs, (uint8_t *)dst_base, recs, tshift, S->btiles[tb], c->base_dev, s);
        }
        // the probe's end mark even when a launch failed: its events go back
        // to the tuner's spares instead of leaking, with no rate
        if (timed) tune_mark(c, zcls, probe, true, s, le == hipSuccess);
        HIP_TRY(le, "launch k_fill_batch");
        HIP_TRY(hipEventRecord(S->filled[tb], s), "hipEventRecord");
        k0 = k1;
    }
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
// The device jump table of lanes sub < lpc starting at draws z0 + sub*span
// (cached per context): jtab[sub] = x^(z0 + sub*span) mod P.
static int jump_table(s3dg_ctx *c, uint32_t lpc, uint64_t span, uint64_t z0, const uint64_t **jtab) {
    std::lock_guard<std::mutex> g(c->mu);
    const std::pair<uint64_t, uint64_t> key{((uint64_t)lpc << 32) | span, z0};
    auto it = c->jtabs.find(key);
    if (it == c->jtabs.end()) {
        // x^(z0 + k*span) = x^(z0 + (k-1)*span) * x^span: one product mod P
        // per lane (a 512-lane table in ~5 ms on the host; round 4 raised a
        // power per lane with bit-wise products, 3 ms each: ~1.6 s on the
        // first small-object DG1 or K2 call of a context)
        std::vector<uint64_t> h(4 * (size_t)lpc, 0);
        uint64_t S[4];
        if (!jump_poly(z0, &h[0]) || !jump_poly(span, S))
            return fail(S3DG_EINVAL, "xoshiro characteristic polynomial unavailable");
        for (uint32_t k = 1; k < lpc; ++k) jump_mul(&h[4 * (k - 1)], S, &h[4 * k]);
        uint64_t *d = nullptr;
        HIP_TRY(hipMalloc(&d, h.size() * 8), "hipMalloc(jump table)");
        HIP_TRY(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice), "hipMemcpy(jump table)");
        it = c->jtabs.emplace(key, d).first;
    }
    *jtab = it->second;
    return S3DG_OK;
}

// z0 > 0: the lanes cover draws [z0, chunk_bytes / 8) of every chunk (the
// tails of a DG1 zero-prefix split), one wave per tail when it has >= 64 x 256 draws.
static int keystream_plan(s3dg_ctx *c, int mode, uint64_t chunk_bytes, uint64_t nchunks, bool zero_prefix,
                          KeystreamArgs &A, const uint64_t **jtab, uint64_t z0 = 0) {
    const uint64_t nd = chunk_bytes / 8 - z0;
    // as many lanes per chunk as keep >= ks_min_draws draws per lane (the
    // jump costs 256 steps); up to 1024 lanes = 16 waves per chunk
    uint64_t min_draws = c->ks_min_draws[mode];
    if (mode == 1 && zero_prefix && min_draws == kDefaultKsMinDraws[1]) min_draws = kDgenPrefixMinDraws;
    if (mode == 0 && min_draws == kDefaultKsMinDraws[0] && nd >= 64 * kKsLongDraws) {
        // waves at 4096 draws per lane vs the chip's resident keystream waves
        // (4 per CU: 64-draw stages take 33 KiB of LDS per wave)
        const uint64_t waves = nchunks * (nd / kKsLongDraws) / 64;
        if (waves >= kKsLongRounds * (uint64_t)c->cus * 4) min_draws = kKsLongDraws;
    }
    uint32_t lpc = 1;
    while (lpc < 1024 && nd / (2 * lpc) >= min_draws) lpc *= 2;
    // a tail: 64 lanes (one wave, the jump's state sequence on the scalar unit)
    if (z0 && lpc < 64 && nd >= 64 * kKsMinSpan) lpc = 64;
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
    A.z0 = z0;
    return jump_table(c, lpc, span, z0, jtab);
}

// The stream's queue counters for persistent keystream launches, allocated
// and zeroed on the stream's first keystream launch.  Caller holds S->mu.
static int ks_counters(StreamState *S, KsCounters **out) {
    if (!S->ks.dev) {
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, kKsCtrBytes), "hipMalloc(keystream counters)");
        const hipError_t e = hipMemset(p, 0, kKsCtrBytes);
        if (e != hipSuccess) {
            (void)hipFree(p);
            HIP_TRY(e, "hipMemset(keystream counters)");
        }
        S->ks.dev = (uint64_t *)p;
        S->ks.par = 0;
    }
    *out = &S->ks;
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
    if (int r = keystream_plan(c, 0, chunk_bytes, (len + chunk_bytes - 1) / chunk_bytes, false, A, &jt)) return r;
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
    StreamLock SL(c, (hipStream_t)stream);
    KsCounters *kc = nullptr;
    if (int r = ks_counters(SL.get(), &kc)) return r;
    HIP_TRY(launch_keystream((uint8_t *)dst, A, jt, c->ks[0], (hipStream_t)stream, kc, c->cus, c->ks_persist),
            "launch k_keystream");
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

int s3dg_dgen_fill_stream(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride, uint64_t n_objs,
                          uint64_t dedup, uint32_t f_num, uint32_t f_den, uint64_t seed_base,
                          uint64_t first_obj, void *stream) {
    if (n_objs > 1 && stride < obj_size) return fail(S3DG_EINVAL, "stride < obj_size: objects overlap");
    return s3dg_internal_dgen_chunk(c, dst, obj_size, stride, n_objs, 0, ~0ull, dedup, f_num, f_den, seed_base,
                                    first_obj, stream);
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
    // zero prefix + tail split: every block of the launch full length, the
    // prefix at least 8 whole granules, enough blocks to pay for two launches
    uint64_t split;
    LaunchCfg zlc;
    bool overlap;
    {
        const int k = (kDgenBlock * f_num) % f_den == 0 && (kDgenBlock * f_num / f_den) % 64 == 0 ? 0 : 1;
        std::lock_guard<std::mutex> g(c->mu);
        split = c->dgen_zero_split;
        zlc.store = c->zp_store >= 0 ? c->zp_store : kZeroPrefixStore[k];
        zlc.waves_per_block = c->zp_waves > 0 ? c->zp_waves : kZeroPrefixWaves[k];
        zlc.dyn_lds = occupancy_lds(c->zp_occ >= 0 ? c->zp_occ : kZeroPrefixOcc[k], 0);
        overlap = (c->zp_overlap >= 0 ? c->zp_overlap : kZeroPrefixOverlap[k]) != 0;
    }
    // the zero launch writes each block's whole 4 KiB granules of zeros (zw
    // bytes); the tail launch starts at draw z0 = zw / 8 and zeroes the rest
    // of the prefix (< 4 KiB) in its lane rows.  Tails that start inside a
    // granule (zw down to 16 B) ran 25-35 % slower: lane regions off the
    // 128-B lines (profiles/r05/g).
    const uint64_t nchunks = (blk_hi - blk_lo) * n_objs;
    const uint32_t zw = (uint32_t)(kDgenBlock * f_num / f_den) & ~(kBlk - 1);
    const bool ragged_end = obj_size % kDgenBlock != 0 && blk_hi == nb;
    if (f_num > 0 && split && ragged_end && blk_hi - 1 > blk_lo && (blk_hi - 1 - blk_lo) * n_objs >= split &&
        zw >= 8 * kBlk) {
        // the objects' full blocks split, their short last blocks in a launch of their own
        if (int r = s3dg_internal_dgen_chunk(c, dst, obj_size, stride, n_objs, blk_lo, blk_hi - 1, dedup, f_num, f_den,
                                             seed_base, first_obj, stream))
            return r;
        return s3dg_internal_dgen_chunk(c, (uint8_t *)dst + (blk_hi - 1 - blk_lo) * kDgenBlock, obj_size, stride,
                                        n_objs, blk_hi - 1, blk_hi, dedup, f_num, f_den, seed_base, first_obj, stream);
    }
    const bool zsplit = f_num > 0 && split && nchunks >= split && zw >= 8 * kBlk && !ragged_end;
    KeystreamArgs A{};
    const uint64_t *jt = nullptr;
    if (int r = keystream_plan(c, 1, kDgenBlock, nchunks, f_num > 0 && !zsplit, A, &jt, zsplit ? zw / 8 : 0))
        return r;
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
    KsShape sh = c->ks[1];
    if (f_num > 0 && !zsplit) {   // zero-prefix launches (512-draw lanes): 4-wave workgroups, groups of 32 waves
        if (c->ks_auto_waves[1]) sh.waves = kDgenPrefixWaves;
        if (c->ks_auto_xcd[1]) sh.xcd_waves = kDgenPrefixXcdWaves;
    }
    StreamLock SL(c, (hipStream_t)stream);
    KsCounters *kc = nullptr;
    if (int r = ks_counters(SL.get(), &kc)) return r;
    hipStream_t s = (hipStream_t)stream;
    StreamState *SS = SL.get();
    // An error after the side stream's zero launch was queued must not return
    // while that launch may still write the caller's buffer (the caller's
    // stream never got to wait on zjoin): drain the side stream first.
    struct ZeroJoinGuard {
        hipStream_t zs = nullptr;
        ~ZeroJoinGuard() {
            if (zs) (void)hipStreamSynchronize(zs);
        }
    } zguard;
    if (zsplit && !overlap) {   // the prefixes' whole granules first (the tail launch masks a partial one)
        HIP_TRY(launch_zero_prefix((uint8_t *)dst, nchunks, A.cpo, stride, kDgenBlock, zw, zlc, s),
                "launch k_zero_prefix");
    } else if (zsplit) {        // on the side stream, concurrent with the tails (disjoint bytes)
        if (!SS->zs) HIP_TRY(hipStreamCreateWithFlags(&SS->zs, hipStreamNonBlocking), "hipStreamCreate(zero)");
        for (hipEvent_t *e : {&SS->zfork, &SS->zjoin})
            if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
        HIP_TRY(hipEventRecord(SS->zfork, s), "hipEventRecord");
        HIP_TRY(hipStreamWaitEvent(SS->zs, SS->zfork, 0), "hipStreamWaitEvent");
        zguard.zs = SS->zs;   // from here an error return first drains the side stream
        HIP_TRY(launch_zero_prefix((uint8_t *)dst, nchunks, A.cpo, stride, kDgenBlock, zw, zlc, SS->zs),
                "launch k_zero_prefix");
        HIP_TRY(hipEventRecord(SS->zjoin, SS->zs), "hipEventRecord");
    }
    // One object: its last T chunks in lanes of half the length, handed out
    // after the others by a persistent launch, so the launch drains on units
    // half as long (default T: half a resident round of 1-wave units, i.e. one
    // round of half units).
    KeystreamArgs A2{};
    const uint64_t *jt2 = nullptr;
    bool tail = false;
    int64_t tail_chunks;
    {
        std::lock_guard<std::mutex> g(c->mu);
        tail_chunks = c->ks_tail;
    }
    if (tail_chunks < 0) {
        int res = 0;
        if (keystream_occupancy(sh, &res) != hipSuccess) res = 0;
        (void)hipGetLastError();
        tail_chunks = (int64_t)((uint64_t)res * (uint64_t)c->cus * (uint64_t)sh.waves * 64 / A.lpc / 2);
    }
    const uint32_t span2 = A.span / 2;
    if (n_objs == 1 && tail_chunks > 0 && sh.waves == 1 && A.lpc >= 64 && A.lpc <= 512 && span2 >= kKsMinSpan &&
        span2 % (uint32_t)sh.draws == 0 && nchunks >= 8 * (uint64_t)tail_chunks) {
        const uint64_t T = (uint64_t)tail_chunks;
        A2 = A;
        A2.lpc = 2 * A.lpc;
        A2.span = span2;
        A2.nchunks = T;
        A2.cpo = T;
        A2.chunk0 = A.chunk0 + (nchunks - T);
        A2.doff = (nchunks - T) * kDgenBlock;
        A.nchunks = nchunks - T;
        A.cpo = nchunks - T;
        if (int r = jump_table(c, A2.lpc, A2.span, A2.z0, &jt2)) return r;
        tail = true;
    }
    HIP_TRY(launch_keystream((uint8_t *)dst, A, jt, sh, s, kc, c->cus, c->ks_persist, tail ? &A2 : nullptr, jt2),
            "launch k_keystream(dgen)");
    if (zsplit && overlap) HIP_TRY(hipStreamWaitEvent(s, SS->zjoin, 0), "hipStreamWaitEvent");
    zguard.zs = nullptr;   // joined: the caller's stream now orders after the zero launch
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
    StreamLock SL(c, s);
    StreamState *S = SL.get();
    if (int r = tiles_reserve(S, nthr, s)) return r;
    HIP_TRY(launch_write_ceiling(cfg_for(c, true), (uint8_t *)dst, len, pattern, S->tiles, nthr, s),
            "launch k_write_ceiling(tiled)");
    return S3DG_OK;
}

int s3dg_write_ceiling_fill(s3dg_ctx *c, void *dst, uint64_t len, uint32_t pace, void *stream) {
    CTX_SCOPE(c);
    if (!dst || !aligned16(dst) || (len % kBlk))
        return fail(S3DG_EINVAL, "dst must be 16-byte aligned and len a multiple of 4096");
    if (len == 0) return S3DG_OK;
    hipStream_t s = (hipStream_t)stream;
    // the tiled fill's launch for len bytes as 8 MiB objects (d1 c1 prefix
    // parameters; one object when len < 8 MiB)
    constexpr uint64_t kObj = 8ull << 20;
    if (len > kObj && len % kObj) return fail(S3DG_EINVAL, "len must be < 8 MiB or a multiple of 8 MiB");
    const uint64_t n_objs = (len + kObj - 1) / kObj;
    const uint64_t obj = len < kObj ? len : kObj;
    PrefixParams pp;
    if (int r = make_prefix(obj / kBlk, 1, 0, 1, &pp)) return r;
    const uint32_t lead = (uint32_t)(((uintptr_t)dst >> 12) & 7);
    const uint32_t tshift = kTileShiftMax;
    const uint64_t tpo = (obj / kBlk + lead + (1ull << tshift) - 1) >> tshift;
    StreamLock SL(c, s);
    StreamState *S = SL.get();
    if (int r = tiles_reserve(S, n_objs * tpo, s)) return r;
    LaunchCfg lc = cfg_for(c, true);
    lc.pace = pace;
    HIP_TRY(launch_fill_uniform_tiles_ablated(lc, (uint8_t *)dst, obj, kObj, n_objs, (uint32_t)tpo,
                                              tshift, lead, pp, S->tiles, c->base_dev, s),
            "launch k_fill_batch(ablated)");
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
    pinned_register(*out, bytes);   // kernels may store into it directly (s3dg_host.cpp small calls)
    return S3DG_OK;
}

int s3dg_host_free_pinned(void *p) {
    pinned_unregister(p);
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
    const int r = s3dg_stream_release(c, stream);
    std::string first = r ? s3dg_last_error() : "";
    const hipError_t e = hipStreamDestroy((hipStream_t)stream);   // even when the drain failed
    if (r) return fail(r, first.c_str());
    HIP_TRY(e, "hipStreamDestroy");
    return S3DG_OK;
}

int s3dg_sync(s3dg_ctx *c, void *stream) {
    CTX_SCOPE(c);
    if (stream) HIP_TRY(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
    else HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return S3DG_OK;
}

}  // extern "C"

extern "C" int s3dg_internal_fail(int code, const char *msg) { return fail(code, msg); }
