// s3dg_kernels.hip — CDNA4 (gfx950) kernels for s3dlio's synthetic payload
// generator.  Semantics: /root/reference/src/data_gen.rs:151-224
// (fill_controlled_data), bit-exact for a given entropy and base block.
//
// Work decomposition (measurements in profiles/):
//   * ONE workgroup per 4 KiB block, non-persistent grid in address order:
//     2 waves per block for streams (each lane two 16-byte stores), 1 wave
//     for batches (four).  Short-lived workgroups dispatched in order keep
//     the write frontier compact; persistent or looping workgroups stayed at
//     5.0-6.3 TB/s on MI355X.
//   * Resident workgroups per CU are capped through reserved LDS (stream:
//     14); fewer blocks in flight write HBM faster than the hardware maximum.
//     Batch workgroups warm the L2 with a later tile record instead.
//   * Stores are global_store_dwordx4 ... sc1: the line leaves the XCD's L2
//     once written (plain stores keep it), measured 2-4 % faster.
//   * Wave 0 derives the block's parameters (u = i % U, zero-prefix length,
//     window offsets) and runs the block's PRNG chain ONCE (SplitMix64 seed
//     words on the VALU, the 8 Xoshiro256++ steps on the scalar unit), then
//     patches the zero bytes and the two 32-byte windows into an LDS image of
//     the base block.  After a barrier every lane stores its 16-byte pieces
//     (zeros below the prefix, the image above).  No HBM reads: dedup blocks
//     are recomputed, never copied.
#include "s3dg_internal.h"

#include <cstdlib>
#include <map>
#include <mutex>

// Diagnostic builds only (tools/ablate.py): bit 0 = no window patch phase,
// bit 1 = no PRNG chain; k_keystream: bit 5 = no Xoshiro steps in the draw
// loop (counter draws), bit 6 = no jump-ahead.  Outputs of such builds are
// wrong by design.
#ifndef S3DG_ABLATE
#define S3DG_ABLATE 0
#endif
// Diagnostic builds only: S3DG_KS_TRACE = per-wave wall-clock stamps of
// k_keystream; S3DG_KS_JUMP bit 0 = per-lane vector jump even when the wave's
// lanes share a chunk (A/B; outputs identical).
#ifndef S3DG_KS_TRACE
#define S3DG_KS_TRACE 0
#endif
#ifndef S3DG_KS_JUMP
#define S3DG_KS_JUMP 0
#endif


namespace s3dg {
#if S3DG_KS_TRACE
// Diagnostic builds only: per-wave start/end wall-clock stamps of k_keystream
// (tools/ks_trace_lab.py).
__device__ uint64_t *g_ks_trace;
#endif
namespace {

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


// 64-bit rotate as two v_alignbit_b32 (the compiler emits shifts + ors):
//   alignbit(a, b, s) = low 32 bits of ((a:b) >> s)
template <int K>
__device__ __forceinline__ uint64_t rotlk(uint64_t x) {
    static_assert(K > 0 && K < 64 && K != 32, "rotate amount");
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (K > 32) { const uint32_t t = lo; lo = hi; hi = t; }
    constexpr int k = K & 31;
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - k);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - k);
    return ((uint64_t)nhi << 32) | nlo;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) {
    return (x << k) | (x >> (64 - k));
}

// SplitMix64 step — SmallRng::seed_from_u64 expansion.
__device__ __forceinline__ uint64_t splitmix_next(uint64_t &x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Xoshiro {
    uint64_t s0, s1, s2, s3;
    __device__ __forceinline__ uint64_t next() {
        const uint64_t r = rotl64(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl64(s3, 45);
        return r;
    }
};

// 16-byte store with a cache policy (LaunchCfg::store; tools/store_lab.py):
//   kStorePlain  global_store_dwordx4 (line kept in the XCD's L2)
//   kStoreNT     ... nt  (__builtin_nontemporal_store)
//   kStoreSC1    ... sc1 (line dropped from the L2 once written)
//   kStoreNTSC1  ... nt sc1
template <int SP>
__device__ __forceinline__ void store16(uint8_t *p, u32x4 v) {
    if constexpr (SP == kStoreNT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    // hipcc neither models nor pads an asm store: a 16-byte store's data
    // registers must not be overwritten for 2 wait states after it issues
    // (cdna_hip_programming.md §5.7), so the pad is inside the string.
    else if constexpr (SP == kStoreSC1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (SP == kStoreNTSC1)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else *reinterpret_cast<u32x4 *>(p) = v;
}

__device__ __forceinline__ uint32_t fastmod(uint32_t a, uint64_t M, uint32_t d) {
    const uint64_t low = M * a;
    return (uint32_t)__umul64hi(low, (uint64_t)d);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {   // SplitMix64 output function
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Per-workgroup LDS: the 4 KiB block image being assembled + its metadata.
struct BlockLds {
    uint8_t img[kBlk];
    uint32_t meta[4];        // c, L
};

// Wave 0, phase 1: block parameters + PRNG chain.  Writes the metadata to LDS
// (lane 0) and returns the window words in `w1`/`w2w` (wave-uniform).
// Scalar-unit budget matters (one SALU per cycle per CU, ~365 cycles per
// 4 KiB block at the write ceiling): the SplitMix64 expansion (all of the
// 64-bit multiplies) runs on the VALU, one seed word per lane; only the 8
// Xoshiro256++ steps (shifts/xors/adds) run on the scalar unit.
struct Plan {
    uint32_t c, L, m, so;
    bool w2;
    uint64_t w1[4], w2w[4];
};

template <bool ABL = false>
__device__ __forceinline__ void plan_block(Plan &P, uint32_t lane, uint32_t i, uint64_t size,
                                           uint64_t entropy, const PrefixParams &pp) {
    const uint32_t u = pp.unique == 0xFFFFFFFFu ? i : fastmod(i, pp.m_unique, pp.unique);  // :201
    const uint64_t off = (uint64_t)i * kBlk;
    const uint32_t L = (uint32_t)((size - off) < kBlk ? (size - off) : kBlk);
    P.L = L;
    if (pp.f_den == 0) {
        // generate_random_data layout (src/data_gen.rs:102-132): no zero prefix,
        // first min(32, L) bytes, then the last 32 bytes when L > HALF_BLK
        P.c = 0;
        P.m = L < kMod ? L : kMod;
        P.so = L - kMod;
        P.w2 = L > kHalf;
    } else {
        uint32_t cl = pp.floor_len;
        if (pp.rem) {                     // closed form of :177-190; period f_den in u
            const uint32_t up = fastmod(u, pp.m_fden, pp.f_den);
            const uint32_t r0 = pp.f_den <= 65536u ? fastmod(up * pp.rem, pp.m_fden, pp.f_den)
                                                   : (uint32_t)(((uint64_t)up * pp.rem) % pp.f_den);
            cl += (uint32_t)((uint64_t)r0 + pp.rem >= pp.f_den);
        }
        P.c = cl < L ? cl : L;                                           // :209
        P.m = (L - P.c) < kMod ? (L - P.c) : kMod;                       // :212-214
        P.so = P.c > kHalf ? P.c : kHalf;                                // :218
        P.w2 = P.m > 0 && P.so + P.m <= L;                               // :219
    }

    // SmallRng::seed_from_u64(u + entropy) (:202-203): state word k =
    // mix64(seed + (k+1)*phi) — lanes 0..3 compute one word each.
    const uint64_t seed = (uint64_t)u + entropy;
    if constexpr (ABL) return;
#if S3DG_ABLATE & 2
    for (int q = 0; q < 4; ++q) { P.w1[q] = seed + q; P.w2w[q] = seed - q; }
    return;
#endif
    Xoshiro g;
#if S3DG_ABLATE & 16
    g.s0 = mix64(seed + 1 * 0x9E3779B97F4A7C15ull);
    g.s1 = mix64(seed + 2 * 0x9E3779B97F4A7C15ull);
    g.s2 = mix64(seed + 3 * 0x9E3779B97F4A7C15ull);
    g.s3 = mix64(seed + 4 * 0x9E3779B97F4A7C15ull);
#else
    const uint64_t zl = mix64(seed + (uint64_t)((lane & 3) + 1) * 0x9E3779B97F4A7C15ull);
    g.s0 = readlane64(zl, 0);
    g.s1 = readlane64(zl, 1);
    g.s2 = readlane64(zl, 2);
    g.s3 = readlane64(zl, 3);
#endif
#if S3DG_ABLATE & 8
    asm volatile("" : "+v"(g.s0), "+v"(g.s1), "+v"(g.s2), "+v"(g.s3));
#endif
    uint64_t r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = g.next();
    if (P.m == kMod) {                // every full block with c <= 4064
#pragma unroll
        for (int q = 0; q < 4; ++q) { P.w1[q] = r[q]; P.w2w[q] = r[4 + q]; }
    } else {
        // fill_bytes_via_next on m < 32 bytes: k1 draws per window, the last
        // one >>32 (next_u32) when its tail is 1..4 bytes
        const uint32_t k1 = (P.m + 7) >> 3;
        const uint32_t tail = P.m & 7;
        const bool tail_hi = tail >= 1 && tail <= 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            P.w1[q] = r[q];
            P.w2w[q] = k1 == 4 ? r[4 + q] : (k1 == 3 ? r[3 + q] : (k1 == 2 ? r[2 + q] : r[1 + q]));
            if (tail_hi && (uint32_t)q + 1 == k1) { P.w1[q] >>= 32; P.w2w[q] >>= 32; }
        }
    }
}

// Byte q (0..31) of a window given as 4 little-endian words.
__device__ __forceinline__ uint8_t window_byte(const uint64_t (&w)[4], uint32_t q) {
    const uint32_t k = (q >> 3) & 3;
    const uint64_t x = k == 0 ? w[0] : (k == 1 ? w[1] : (k == 2 ? w[2] : w[3]));
    return (uint8_t)(x >> (8 * (q & 7)));
}

// Wave 0, phase 2 (after every lane has copied the base block into the image):
// zero bytes [c & ~15, c) of the partial segment, then window 1 at c, then
// window 2 at so (later write wins, as :217-221).  One byte per lane.
__device__ __forceinline__ void patch_image(BlockLds &S, const Plan &P, uint32_t lane) {
    const uint32_t z0 = P.c & ~15u;
    if (lane < P.c - z0) S.img[z0 + lane] = 0;                           // :209-210
    if (lane < P.m) S.img[P.c + lane] = window_byte(P.w1, lane);         // :217
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (P.w2 && lane < P.m) S.img[P.so + lane] = window_byte(P.w2w, lane);   // :219-221
}

// Every lane, phase 3: its 16 bytes at byte o of the block: zeros below c, else the image.
// Diagnostic builds only (tools/variant_lab.py, config-3 A/Bs): S3DG_DIAG_ZERO
// bit 0 = zero-prefix pieces store the constant S3DG_DIAG_ZVAL instead of 0
// (same instructions, other data; wrong bytes by design), bit 1 = zero-prefix
// pieces read their LDS image piece too (same data, the store stream paced
// like a prefix-free block), bit 2 = a block's pieces stored last-first;
// S3DG_DIAG_ZPOL = store policy of the zero-prefix pieces (kStore*).
#ifndef S3DG_DIAG_ZERO
#define S3DG_DIAG_ZERO 0
#endif
#ifndef S3DG_DIAG_ZVAL
#define S3DG_DIAG_ZVAL 0x5A5A5A5Au
#endif
template <int NT>
__device__ __forceinline__ void write_block(uint8_t *bd, const BlockLds &S, int o) {
    const int c = (int)S.meta[0], L = (int)S.meta[1];
    if (o >= L) return;
#if S3DG_DIAG_ZERO & 1
    const u32x4 zero = {S3DG_DIAG_ZVAL, S3DG_DIAG_ZVAL, S3DG_DIAG_ZVAL, S3DG_DIAG_ZVAL};
#else
    const u32x4 zero = {0u, 0u, 0u, 0u};
#endif
#if S3DG_DIAG_ZERO & 2
    u32x4 im = *reinterpret_cast<const u32x4 *>(S.img + o);
    asm volatile("" : "+v"(im));
    const u32x4 v = (o + 16 <= c) ? zero : im;
#else
    const u32x4 v = (o + 16 <= c) ? zero : *reinterpret_cast<const u32x4 *>(S.img + o);
#endif
    if (o + 16 <= L) {
#ifdef S3DG_DIAG_ZPOL
        if (o + 16 <= c) store16<S3DG_DIAG_ZPOL>(bd + o, v);   // diagnostic: zero pieces' own store policy
        else
#endif
        store16<NT>(bd + o, v);
    } else {                                  // ragged object tail: bytes < L only
        const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
        for (int b = 0; b < 16 && o + b < L; ++b)
            bd[o + b] = (uint8_t)(dw[b >> 2] >> (8 * (b & 3)));
    }
}

// The whole per-block body (all three phases); NW waves per 4 KiB block.
// Base-block pieces of thread t (issued first: they depend on kernel
// arguments only, so their latency overlaps the plan's inputs).
template <int NW>
__device__ __forceinline__ void load_base(u32x4 (&B)[4 / NW], uint32_t t, const u32x4 *base) {
    constexpr int T = 64 * NW;
#pragma unroll
    for (int k = 0; k < 4 / NW; ++k) B[k] = base[t + k * T];   // bytes 16(t+kT).. of the base block
}

template <int NW>
__device__ __forceinline__ void store_image(BlockLds &S, uint32_t t, const u32x4 (&B)[4 / NW]) {
    constexpr int T = 64 * NW;
#pragma unroll
    for (int k = 0; k < 4 / NW; ++k)
        *reinterpret_cast<u32x4 *>(S.img + 16 * (t + k * T)) = B[k];   // :205-207
}

// IMG: the caller has already written the base image into S (batch kernel).
// ABL: the store-only reference of the same kernel (write ceiling): block
// geometry, LDS image, barrier and stores as the fill, without the PRNG chain
// and the window patch phase; its bytes are wrong by design.
// rt_floor > 0: the block's stores wait until rt_floor wall-clock ticks
// (100 MHz) after its workgroup started (t0): a floor on the time before the
// stores that does not scale with the GFX clock.
template <int NT, int NW, bool IMG = false, bool ABL = false>
__device__ __forceinline__ void gen_block(uint8_t *bd, BlockLds &S, uint32_t t, uint32_t wave,
                                          uint32_t i, uint64_t size, uint64_t entropy,
                                          const PrefixParams &pp, const u32x4 (&B)[4 / NW], uint64_t t0 = 0,
                                          uint32_t rt_floor = 0) {
    constexpr int T = 64 * NW, SPL = 4 / NW;   // segments per lane
    const uint32_t lane = t & 63;
    Plan P;
    if (wave == 0) {
        plan_block<ABL>(P, lane, i, size, entropy, pp);
        if (lane == 0) { S.meta[0] = P.c; S.meta[1] = P.L; }
    }
    if constexpr (!IMG) store_image<NW>(S, t, B);
    __syncthreads();
#if !(S3DG_ABLATE & 1)
    if constexpr (!ABL) {
        if (wave == 0) patch_image(S, P, lane);
        __syncthreads();
    }
#endif
    // bounded as well by sleep count (4 x rt_floor sleeps of >= 64 cycles, i.e.
    // at least rt_floor x 256 cycles), so the wait ends even if the real-time
    // counter did not advance
    if (rt_floor)
        for (uint32_t n = 0; n < 4 * rt_floor && wall_clock64() - t0 < (uint64_t)rt_floor; ++n)
            __builtin_amdgcn_s_sleep(1);
#if S3DG_DIAG_ZERO & 4
    // diagnostic: pieces stored last-first (the zero prefix's stores after the image's)
#pragma unroll
    for (int k = SPL - 1; k >= 0; --k) write_block<NT>(bd, S, (int)(t + k * T) * 16);
#else
#pragma unroll
    for (int k = 0; k < SPL; ++k) write_block<NT>(bd, S, (int)(t + k * T) * 16);
#endif
}

// Stream: blockIdx.x = block (blk_lo + x) of object blockIdx.y of this launch
// (dst and ent0 already advanced to the launch's first object).  Argument
// order matters: the first 14 dwords arrive preloaded in SGPRs, the rest by
// a scalar load from the kernarg segment, so base (needed first) and
// everything up to the plan's first use lead and the prefix parameters trail.
template <int NT, int NW>
__global__ __launch_bounds__(64 * NW) void k_fill_stream(uint8_t *dst, const u32x4 *base, uint64_t stride,
                                                         uint64_t ent0, uint64_t obj_size, uint32_t blk_lo,
                                                         PrefixParams pp) {
    __shared__ __attribute__((aligned(16))) BlockLds S;
    const uint32_t t = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
    uint64_t jv = blockIdx.y;        // block address on the VALU: keep the scalar unit
    asm volatile("" : "+v"(jv));     // for the PRNG chain
    uint8_t *bd = dst + jv * stride + (uint64_t)blockIdx.x * kBlk;
    u32x4 B[4 / NW];
    load_base<NW>(B, t, base);
    gen_block<NT, NW>(bd, S, t, wave, blk_lo + blockIdx.x, obj_size,
                      ent0 + ((uint64_t)blockIdx.y << 32), pp, B);
}

// Batch: workgroup g -> tile record g >> tshift (one scalar load), block
// first + (g mod 2^tshift) - lead of that object; slots before the object's
// start (lead) or past its end exit.  lead makes g = 4 KiB-granule address
// (mod 8), as in the stream kernel: workgroups are dealt round-robin to the
// 8 XCDs, so XCD x writes only granules = x (mod 8).
// Tiles are 2^tshift blocks (2..64, chosen per launch by the host so the
// dead workgroups of ragged object tails stay few).
// pf > 0: the first 8 workgroups of every 256 blocks (one per XCD: workgroups
// are dealt round-robin to the XCDs) touch the records of the 256 blocks
// 64*pf blocks ahead (one lane per 128-byte line of records) after their
// stores, result unused, so they are in that XCD's L2 when its workgroups
// start.  pf must exceed the resident workgroups / 64.
// FLOOR: the fill with the wall-clock floor compiled in (launches whose
// rt_floor > 0).  The floor-free instantiation carries none of its code: the
// conditional real-time read and wait cost launches that never use them
// 0.3-1 % (round 4 library A/B).
template <int NT, int NW, bool ABL = false, bool FLOOR = false>
__global__ __launch_bounds__(64 * NW) void k_fill_batch(uint8_t *dst_base, const TileRec *tiles,
                                                        uint64_t ntiles, uint64_t g0, uint32_t pf,
                                                        uint32_t tshift, const u32x4 *base, uint32_t pace) {
    __shared__ __attribute__((aligned(16))) BlockLds S;
    const uint32_t t = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6);
    // pace: the store-only reference's wave-0 delay (ABL), else the fill's
    // wall-clock floor before the stores (rt_floor; FLOOR instantiation only)
    const uint64_t t0 = (!ABL && FLOOR) ? wall_clock64() : 0;
    const uint64_t g = g0 + blockIdx.x;
    const uint64_t tile = g >> tshift;
    // The tile record (64 B) in ONE scalar load, issued first; then the base
    // block's vector loads and its LDS image, so the two memory latencies
    // overlap instead of following each other (the compiler otherwise splits
    // the record into four loads around the early-exit branch).
    u32x16 raw;
    asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(raw) : "s"(tiles + tile) : "memory");
    u32x4 B[4 / NW];
    load_base<NW>(B, t, base);
    // the wait "redefines" raw, so no use of the record can move above it.
    // The LDS image is written after it (round 4): before, this wait also
    // covered the image's ds_writes, which wait for the base block's loads,
    // so the record-dependent work (and a dead slot's exit) started only once
    // those had landed; after: config 2 +0.45-0.5 %, config 4 +0.2 %,
    // config 3 -0.25 % (two library A/Bs, profiles/r04/d, profiles/r04/e).
    // Later still, after wave 0's plan (gen_block's own image write), lost
    // 3.5-5.7 % on configs 2, 4 and 5 (profiles/r04/g).
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(raw) :: "memory");
    const TileRec e = __builtin_bit_cast(TileRec, raw);
    const uint32_t k = (uint32_t)(g & ((1u << tshift) - 1));
    const int64_t ib = (int64_t)e.first + k - e.lead;
    uint8_t *const bdst = dst_base + e.dst_off + (uint64_t)ib * kBlk;
    if (ib < 0 || (uint64_t)ib * kBlk >= e.size) return;   // uniform for the whole workgroup
    store_image<NW>(S, t, B);
    if constexpr (ABL) {   // store-only reference: wave 0 idles `pace` x 2 x 64 cycles in the plan's place
        if (wave == 0)
            for (uint32_t q = 0; q < pace; ++q) __builtin_amdgcn_s_sleep(2);
    }
    gen_block<NT, NW, true, ABL>(bdst, S, t, wave, (uint32_t)ib, e.size, e.entropy, e.pp, B, t0,
                                 (!ABL && FLOOR) ? pace : 0u);
    // one prefetching workgroup per XCD per span blocks (256: 128 and 512
    // measured slower); lane q of it touches the q-th
    // 128-byte line (2 records) of the span's records
    constexpr uint32_t kPfSpan = 256;
    const uint32_t span = kPfSpan > (2u << tshift) ? kPfSpan : (2u << tshift);
    if (pf && (g & (span - 1)) < 8) {
        const uint64_t first = ((g + 64ull * pf) & ~(uint64_t)(span - 1)) >> tshift;
        if (tshift == 0) {
            // one record per block: this workgroup's XCD (g mod 8, dealt
            // round-robin) uses only the records = g (mod 8) of the span, so
            // it touches those 32 and leaves the rest to the other XCDs
            if (t < span / 8) {
                const uint64_t pt = first + 8 * t + (g & 7);
                const TileRec *p = tiles + (pt < ntiles ? pt : ntiles - 1);
                uint32_t dummy;
                asm volatile("global_load_dword %0, %1, off" : "=v"(dummy) : "v"(p) : "memory");
            }
        } else if (t < (span >> (tshift + 1))) {
            const uint64_t pt = first + 2 * t;
            const TileRec *p = tiles + (pt < ntiles ? pt : ntiles - 1);
            uint32_t dummy;
            asm volatile("global_load_dword %0, %1, off" : "=v"(dummy) : "v"(p) : "memory");
        }
    }
}

// Prefix parameters of one object on the device, as the host's make_prefix
// (src/data_gen.rs:162-175; s3dg_unique_blocks' f64 round half away from zero).
__device__ PrefixParams dev_make_prefix(uint64_t nb, uint64_t dedup, uint32_t f_num, uint32_t f_den) {
    const uint64_t d = dedup == 0 ? 1 : dedup;
    uint64_t U = nb;
    if (d > 1) {
        double r = round((double)nb / (double)d);
        if (r < 1.0) r = 1.0;
        U = (uint64_t)r;
    }
    PrefixParams pp;
    const uint64_t tot = (uint64_t)f_num * kBlk;
    pp.unique = U == nb ? 0xFFFFFFFFu : (uint32_t)U;
    pp.floor_len = (uint32_t)(tot / f_den);
    pp.rem = (uint32_t)(tot % f_den);
    pp.f_den = f_den;
    pp.m_unique = ~0ull / (pp.unique == 0xFFFFFFFFu ? 1u : pp.unique) + 1;
    pp.m_fden = ~0ull / f_den + 1;
    return pp;
}

// Records of a batch sub-batch from its uploaded descriptors, one thread per
// object: record q in [rec_lo, rec_hi) maps slot (q << tshift) + k to block
// (q - rec_lo) << tshift + k - lead.  Tile layouts: rec_lo from the scan, lead
// = the object's granule mod 8 (XCD alignment).  Dense: rec_lo = the object's
// granule slot (0 for the first object, whose lead is lead0), rec_hi = the
// next object's, so the gap records before it are its dead slots.
// An object with few records writes them itself; the records of objects with
// more (a multi-GiB object, a dense layout with large gaps) are written by the
// whole wave, 64 per pass, so no lane loops over tens of thousands of them
// while the fill waits.
constexpr uint64_t kMapOwnRecords = 16;
__global__ __launch_bounds__(256) void k_batch_map(const s3dg_obj_desc *d, uint64_t n, const uint64_t *scan,
                                                   TileRec *tiles, uint32_t tshift, uint64_t base, uint64_t lead0,
                                                   uint64_t first_off) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    TileRec r{};
    uint64_t rec_lo = 0, rec_hi = 0;
    if (k < n) {
        const s3dg_obj_desc o = d[k];
        const uint64_t nb = (o.size + kBlk - 1) / kBlk;
        uint64_t lead;
        if (tshift == 0) {
            const uint64_t g0 = lead0 + (o.dst_off - first_off) / kBlk;
            rec_lo = k == 0 ? 0 : g0;
            rec_hi = k + 1 < n ? lead0 + (d[k + 1].dst_off - first_off) / kBlk : g0 + nb;
            lead = g0 - rec_lo;
        } else {
            lead = ((base + o.dst_off) >> 12) & 7;
            rec_lo = scan[k];
            rec_hi = rec_lo + ((nb + lead + (1ull << tshift) - 1) >> tshift);
        }
        r.dst_off = o.dst_off;
        r.size = o.size;
        r.entropy = o.entropy;
        r.lead = (uint32_t)lead;
        r.pp = dev_make_prefix(nb, o.dedup, o.f_num, o.f_den);
    }
    const bool own = rec_hi - rec_lo <= kMapOwnRecords;
    if (own)
        for (uint64_t q = rec_lo; q < rec_hi; ++q) {
            r.first = (uint32_t)((q - rec_lo) << tshift);
            tiles[q] = r;
        }
    // the wave's objects with many records, one after the other, 64 records per pass
    uint64_t big = __ballot(!own);
    while (big) {
        const int src = __builtin_ctzll(big);
        big &= big - 1;
        TileRec b;
        uint32_t *bw = reinterpret_cast<uint32_t *>(&b);
        const uint32_t *rw = reinterpret_cast<const uint32_t *>(&r);
#pragma unroll
        for (int w = 0; w < 16; ++w) bw[w] = __builtin_amdgcn_readlane(rw[w], src);
        const uint64_t lo = readlane64(rec_lo, src), hi = readlane64(rec_hi, src);
        for (uint64_t q = lo + lane; q < hi; q += 64) {
            b.first = (uint32_t)((q - lo) << tshift);
            tiles[q] = b;
        }
    }
}

// tiles[q] for a uniform stream: n objects of obj_size bytes at dst_off =
// j * stride, entropy ent0 + (j << 32), all with the same lead (stride a
// multiple of 32 KiB), tiles_per_obj tiles each.
__global__ __launch_bounds__(256) void k_tile_map_uniform(TileRec *tiles, uint64_t ntiles, uint32_t tiles_per_obj,
                                                          uint32_t tshift, uint64_t stride, uint64_t obj_size,
                                                          uint64_t ent0, uint32_t lead, PrefixParams pp) {
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= ntiles) return;
    const uint64_t j = q / tiles_per_obj;
    TileRec r;
    r.dst_off = j * stride;
    r.size = obj_size;
    r.entropy = ent0 + (j << 32);
    r.first = (uint32_t)((q - j * tiles_per_obj) << tshift);
    r.lead = lead;
    r.pp = pp;
    tiles[q] = r;
}

// Write-only ceiling in the fill kernels' shape: one 4 KiB chunk per
// (64*NW)-thread workgroup, 16-byte stores, same occupancy cap.  pf > 0:
// the tiled fill's trailing loads too (64-block records in thr, 256-block
// spans, k_fill_batch), so the ceiling covers that shape.
template <int NT, int NW>
__global__ __launch_bounds__(64 * NW) void k_write_ceiling(uint8_t *dst, uint64_t nchunks, uint64_t g0,
                                                           uint32_t pat, const TileRec *thr, uint64_t nthr,
                                                           uint32_t pf) {
    const u32x4 v = {pat, pat ^ 0x9E3779B9u, pat + 1u, ~pat};
    const uint64_t g = g0 + blockIdx.x;
    if (g >= nchunks) return;
#pragma unroll
    for (int k = 0; k < 4 / NW; ++k) store16<NT>(dst + g * kBlk + (threadIdx.x + k * 64 * NW) * 16, v);
    if (pf && (g & 255) < 8 && threadIdx.x < 2) {
        const uint64_t pt = (((g + 64ull * pf) & ~255ull) >> 6) + 2 * threadIdx.x;
        const TileRec *p = thr + (pt < nthr ? pt : nthr - 1);
        uint32_t dummy;
        asm volatile("global_load_dword %0, %1, off" : "=v"(dummy) : "v"(p) : "memory");
    }
}


// ---------------------------------------------------------------------------
// K2: keystream fill (generate_npz_bytes_raw x-fill, src/data_formats/npz.rs:376-383).
// Chunk c (chunk_bytes each, last one ragged) of [dst, dst+len) =
//   Xoshiro256PlusPlus::seed_from_u64(seed_base + c).fill_bytes(chunk).
// `lpc` lanes share a chunk: lane `sub` starts at draw sub*span via the
// jump polynomial jtab[sub] = x^(sub*span) mod P (s3dg_jump.cpp), 256 steps.
// Each iteration a lane makes D draws (8D bytes) into its LDS row; the wave
// then writes the 64 rows out with 16-byte pieces, P = D/2 pieces per row and
// 64/P rows per store instruction, so every store covers whole 8D-byte row
// segments (D = 16: 128 B, 8 rows per instruction; D = 64: 512 B, 2 rows).
// W waves per workgroup; LDS = W * 64 * (8D + 16) bytes.
// a ^ b ^ c on 64-bit lanes: two v_bitop3_b32 (gfx950 3-input LUT op, 0x96 =
// XOR3) instead of four v_xor_b32; the compiler does not form it itself.
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)a, (uint32_t)b, (uint32_t)c, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(a >> 32), (uint32_t)(b >> 32),
                                                    (uint32_t)(c >> 32), 0x96);
    return ((uint64_t)hi << 32) | lo;
}

// a ^ (s & m) with a 32-bit mask m applied to both halves: v_bitop3 0x6C =
// S1 ^ (S0 & S2) (symmetric in S0, S2, so independent of the LUT's bit order).
__device__ __forceinline__ uint64_t and_xor_64(uint64_t s, uint64_t a, uint32_t m) {
    const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)s, (uint32_t)a, m, 0x6C);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(s >> 32), (uint32_t)(a >> 32), m, 0x6C);
    return ((uint64_t)hi << 32) | lo;
}

// Xoshiro256++ output rotl(s0 + s3, 23) + s0.  The empty asm pins the
// rotated value as one 64-bit register pair; without it the compiler turns
// the rotate's OR of two disjoint halves into two adds plus two moves.
__device__ __forceinline__ uint64_t xo_out(uint64_t s0, uint64_t s3) {
    uint64_t r = rotlk<23>(s0 + s3);
    asm("" : "+v"(r));
    return r + s0;
}

// One Xoshiro256 state step (per lane, VALU): the reference order
// s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45)
// with the chained XORs folded into 3-input ones (11 VALU ops, was 13).
__device__ __forceinline__ void xo_step(uint64_t &s0, uint64_t &s1, uint64_t &s2, uint64_t &s3) {
    const uint64_t t = s1 << 17;
    const uint64_t n1 = xor3_64(s1, s2, s0);
    const uint64_t n0 = xor3_64(s0, s3, s1);
    const uint64_t n2 = xor3_64(s2, s0, t);
    s3 = rotlk<45>(s3 ^ s1);
    s0 = n0; s1 = n1; s2 = n2;
}

// Workgroups are dealt round-robin to the 8 XCDs, so consecutive ones write
// through different L2s.  Each full group of 8*xg workgroups is remapped so
// the xg workgroups one XCD receives take xg adjacent work units: every XCD
// writes runs of xg*W*64 adjacent lane regions (the last,
// partial group keeps the dealing order).  b: the workgroup's index in the
// static grid of A.nwg workgroups (dealt to XCD b mod 8).
__device__ __forceinline__ uint64_t ks_remap(const KeystreamArgs &A, uint64_t b) {
    if (A.xg > 1) {
        const uint32_t gs = (uint32_t)__builtin_ctz(A.xg);
        if (((b >> (gs + 3)) + 1) << (gs + 3) <= A.nwg) {
            const uint64_t x = b & 7, k = b >> 3;
            return ((k >> gs) << (gs + 3)) + (x << gs) + (k & (A.xg - 1));
        }
    }
    return b;
}

// One work unit: wave w of remapped workgroup bid, i.e. lanes
// [(bid*W + w)*64, +64) of the launch.  myrows: this wave's LDS rows.
template <int D, int W, int SP>
__device__ __forceinline__ void ks_unit(uint8_t *dst, const KeystreamArgs &A, const uint64_t *jtab,
                                        uint8_t *myrows, uint32_t l, uint64_t bid, uint32_t w) {
    static_assert(D == 16 || D == 32 || D == 64, "draws per stage");
    constexpr int RS = D * 8 + 16;     // row stride: + 16 B pad, conflict-light ds_write_b128 rows
    constexpr int P = D / 2;           // 16-byte pieces per row
    constexpr int R = 64 / P;          // rows per store instruction
#if S3DG_KS_TRACE
    const uint64_t t_start = wall_clock64();
#endif
    const uint32_t lpc = A.lpc, span = A.span;
    // global lane gl -> chunk gl / lpc, lane-in-chunk gl % lpc (lpc: power of two;
    // lpc > 64 spreads one chunk over lpc/64 waves)
    const uint32_t lsh = (uint32_t)__builtin_ctz(lpc);
    const uint64_t gl = (bid * W + w) * 64 + l;
    const uint64_t c = gl >> lsh;                                    // local chunk index
    const uint64_t cpo = A.cpo ? A.cpo : A.nchunks;
    const uint64_t ko = c / cpo;                                     // object within the launch
    const uint64_t cl = c - ko * cpo;
    const uint64_t cg = A.chunk0 + cl;                               // chunk index in the object
    const uint32_t sub = (uint32_t)(gl & (lpc - 1));
    const uint64_t coff = A.doff + ko * A.obj_stride + cl * A.chunk_bytes;   // offset within dst
    const uint64_t seed_base = A.seed_base + ko * A.seed_step;
    const uint64_t gofs = cg * A.chunk_bytes;                        // offset within the object
    const uint64_t clen = (c < A.nchunks && gofs < A.obj_len)
                              ? ((A.obj_len - gofs) < A.chunk_bytes ? (A.obj_len - gofs) : A.chunk_bytes)
                              : 0;
    const uint64_t d0 = A.z0 + (uint64_t)sub * span;                 // first draw index
    const uint64_t rb = d0 * 8;                                      // lane region within chunk
    const uint32_t rlen = (uint32_t)(clen > rb ? ((clen - rb) < (uint64_t)span * 8 ? (clen - rb) : (uint64_t)span * 8) : 0);
    const uint64_t tail_draw = clen >> 3;                            // draw index of a 1..7 B tail
    const bool tail_hi = (clen & 7) >= 1 && (clen & 7) <= 4;         // next_u32 = next_u64 >> 32
    // zero prefix of the chunk (dgen-contract compressibility); 0 for the npz fill
    const uint64_t zlen = A.zf_num ? (clen * A.zf_num) / A.zf_den : 0;

    // chunk seed: npz.rs:381 seed_from_u64(k), or the dgen mode
    // seed ^ (u * phi) with u = chunk % U (dedup)
    uint64_t x;
    if (A.seed_mode == 0) {
        x = seed_base + cg;
    } else {
        const uint32_t u = A.unique == 0xFFFFFFFFu ? (uint32_t)cg : fastmod((uint32_t)cg, A.m_unique, A.unique);
        x = seed_base ^ ((uint64_t)u * 0x9E3779B97F4A7C15ull);
    }
    uint64_t s0 = mix64(x + 0x9E3779B97F4A7C15ull), s1 = mix64(x + 2 * 0x9E3779B97F4A7C15ull);
    uint64_t s2 = mix64(x + 3 * 0x9E3779B97F4A7C15ull), s3 = mix64(x + 4 * 0x9E3779B97F4A7C15ull);
    const uint32_t iters = span / D;
    const uint32_t piece = l % P;
    // destination of the P rows this lane helps write: row R*i + l/P, piece l%P
    uint64_t raddr[P];
    uint32_t rrem[P];
    auto row_dest = [&]() {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            const uint32_t r = R * i + l / P;
            raddr[i] = __shfl(coff + rb, (int)r);
            rrem[i] = __shfl(rlen, (int)r);
        }
    };
    const bool full_rows = __all(rlen == span * 8u);

    // A wave whose regions all lie inside their chunks' zero prefixes (DG1,
    // compress > 1) stores zeros: no jump, no PRNG.
    if (__all(rlen == 0 || rb + rlen <= zlen)) {
        row_dest();
        const u32x4 z = {0u, 0u, 0u, 0u};
        for (uint32_t it = 0; it < iters; ++it) {
            const uint32_t o = it * (D * 8) + piece * 16;
#pragma unroll
            for (int i = 0; i < P; ++i) {
                if (full_rows) {
                    store16<SP>(dst + raddr[i] + o, z);
                } else if (o < rrem[i]) {
                    uint8_t *q = dst + raddr[i] + o;
                    if (o + 16 <= rrem[i]) store16<SP>(q, z);
                    else for (uint32_t b = 0; o + b < rrem[i]; ++b) q[b] = 0;
                }
            }
        }
        return;
    }

#if !(S3DG_ABLATE & 64)
    if (lpc >= 64 && !(S3DG_KS_JUMP & 1)) {
        // Every lane of the wave is in one chunk, so the sequence step^i(s)
        // is wave-uniform: it runs on the scalar unit (64-bit s_xor/s_lshl,
        // SGPRs) and each lane only accumulates the states its own jump
        // polynomial selects (8 v_bitop3 with an SGPR operand per step, was
        // 8 + the 11-op vector step).  Lane sub = 0 of a launch with z0 = 0
        // has J = 1: a = s.
        uint64_t u0 = readlane64(s0, 0), u1 = readlane64(s1, 0);
        uint64_t u2 = readlane64(s2, 0), u3 = readlane64(s3, 0);
        // the lane's 256-bit polynomial in two loads up front (one load and
        // wait per 32 steps before)
        const uint4 *Jv = reinterpret_cast<const uint4 *>(jtab + 4 * sub);
        const uint4 j0 = Jv[0], j1 = Jv[1];
        const uint32_t J[8] = {j0.x, j0.y, j0.z, j0.w, j1.x, j1.y, j1.z, j1.w};
        uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const uint32_t jw = J[h];
#pragma unroll 8
            for (int b = 0; b < 32; ++b) {
                const uint32_t m = (uint32_t)((int32_t)(jw << (31 - b)) >> 31);
                a0 = and_xor_64(u0, a0, m); a1 = and_xor_64(u1, a1, m);
                a2 = and_xor_64(u2, a2, m); a3 = and_xor_64(u3, a3, m);
                const uint64_t t = u1 << 17;    // reference step order, scalar
                u2 ^= u0; u3 ^= u1; u1 ^= u2; u0 ^= u3; u2 ^= t;
                u3 = rotl64(u3, 45);
            }
        }
        s0 = a0; s1 = a1; s2 = a2; s3 = a3;
    } else if (A.z0 || (lpc > 1 && sub > 0)) {   // jump to draw z0 + sub*span
        // state <- sum over set bits i of J of step^i(state): 256 steps, the
        // polynomial read as 8 32-bit halves so each step's mask is one
        // sign-extended bit field and each accumulate one v_bitop3
        const uint32_t *J = reinterpret_cast<const uint32_t *>(jtab + 4 * sub);
        uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        for (int h = 0; h < 8; ++h) {
            const uint32_t jw = J[h];
#pragma unroll 4
            for (int b = 0; b < 32; ++b) {
                const uint32_t m = (uint32_t)((int32_t)(jw << (31 - b)) >> 31);
                a0 = and_xor_64(s0, a0, m); a1 = and_xor_64(s1, a1, m);
                a2 = and_xor_64(s2, a2, m); a3 = and_xor_64(s3, a3, m);
                xo_step(s0, s1, s2, s3);
            }
        }
        s0 = a0; s1 = a1; s2 = a2; s3 = a3;
    }
#endif
    row_dest();

    // Wave-uniform fast path: a D-draw group is generated unmasked unless a
    // lane of the wave is at its chunk's 1-4 byte tail (iteration it_tail);
    // bytes inside a zero prefix are then zeroed in the lane's LDS row by the
    // lanes concerned alone (round 5: the whole wave used to take the masked
    // path while any lane touched the prefix, e.g. 6 of 8 store rounds of a
    // DG1 c3 wave, or 8 of 11 of a tail launch's waves, profiles/r05/).  The
    // stores need no guards when every region of the wave is full length.
    const uint32_t it_tail = (tail_hi && tail_draw >= d0 && tail_draw < d0 + span)
                                 ? (uint32_t)((tail_draw - d0) / D) : 0xFFFFFFFFu;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint64_t dg = d0 + (uint64_t)it * D;
        const bool plain = __all(it != it_tail);
        if (plain) {
#pragma unroll
            for (int q = 0; q < D; q += 2) {
#if S3DG_ABLATE & 32
                const uint64_t ra = s0 + q, rbv = s3 + q;
#else
                const uint64_t ra = xo_out(s0, s3); xo_step(s0, s1, s2, s3);
                const uint64_t rbv = xo_out(s0, s3); xo_step(s0, s1, s2, s3);
#endif
                *reinterpret_cast<u32x4 *>(myrows + l * RS + q * 8) =
                    u32x4{(uint32_t)ra, (uint32_t)(ra >> 32), (uint32_t)rbv, (uint32_t)(rbv >> 32)};
            }
        } else {
#pragma unroll
            for (int q = 0; q < D; q += 2) {
                uint64_t ra = xo_out(s0, s3); xo_step(s0, s1, s2, s3);
                uint64_t rbv = xo_out(s0, s3); xo_step(s0, s1, s2, s3);
                const uint64_t d = dg + q;
                if (tail_hi && d == tail_draw) ra >>= 32;
                if (tail_hi && d + 1 == tail_draw) rbv >>= 32;
                if (8 * d < zlen) ra &= (8 * d + 8 <= zlen) ? 0ull : (~0ull << (8 * (zlen - 8 * d)));
                if (8 * d + 8 < zlen) rbv &= (8 * d + 16 <= zlen) ? 0ull : (~0ull << (8 * (zlen - 8 * d - 8)));
                *reinterpret_cast<u32x4 *>(myrows + l * RS + q * 8) =
                    u32x4{(uint32_t)ra, (uint32_t)(ra >> 32), (uint32_t)rbv, (uint32_t)(rbv >> 32)};
            }
        }
        // zero-prefix bytes of this row (fast path only: the masked path zeroed them)
        const uint64_t row0 = 8 * dg;
        if (plain && row0 < zlen) {
            const uint32_t zb = (zlen - row0) < (uint64_t)(D * 8) ? (uint32_t)(zlen - row0) : (uint32_t)(D * 8);
            uint8_t *row = myrows + l * RS;
            for (uint32_t p = 0; p + 16 <= zb; p += 16) *reinterpret_cast<u32x4 *>(row + p) = u32x4{0u, 0u, 0u, 0u};
            if (zb & 15u) {
                u32x4 *pc = reinterpret_cast<u32x4 *>(row + (zb & ~15u));
                u32x4 v = *pc;
                const uint32_t nz = zb & 15u;   // leading bytes to zero
                v.x = nz >= 4 ? 0u : v.x & (~0u << (8 * nz));
                v.y = nz >= 8 ? 0u : nz <= 4 ? v.y : v.y & (~0u << (8 * (nz - 4)));
                v.z = nz >= 12 ? 0u : nz <= 8 ? v.z : v.z & (~0u << (8 * (nz - 8)));
                v.w = nz <= 12 ? v.w : v.w & (~0u << (8 * (nz - 12)));
                *pc = v;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t o = it * (D * 8) + piece * 16;               // offset within the row's region
        if (full_rows) {
            // Pieces are read from LDS a group of 8 ahead of their stores, so
            // each read's latency hides behind the previous group's stores
            // (the compiler otherwise pairs each read with its store and waits
            // P times per stage): +2 % (variant_ksgroup.log).
            constexpr int G = P < 8 ? P : 8;
            u32x4 v[P];
#pragma unroll
            for (int i = 0; i < G; ++i)
                v[i] = *reinterpret_cast<const u32x4 *>(myrows + (R * i + l / P) * RS + piece * 16);
#pragma unroll
            for (int g = 0; g < P; g += G) {
                if (g + G < P) {
#pragma unroll
                    for (int i = g + G; i < g + 2 * G; ++i)
                        v[i] = *reinterpret_cast<const u32x4 *>(myrows + (R * i + l / P) * RS + piece * 16);
                }
                asm volatile("" ::: "memory");
#pragma unroll
                for (int i = g; i < g + G; ++i) store16<SP>(dst + raddr[i] + o, v[i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < P; ++i) {
                const uint32_t r = R * i + l / P;
                if (o >= rrem[i]) continue;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(myrows + r * RS + piece * 16);
                uint8_t *p = dst + raddr[i] + o;
                if (o + 16 <= rrem[i]) {
                    store16<SP>(p, v);
                } else {
                    const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
                    for (uint32_t b = 0; b < 16 && o + b < rrem[i]; ++b) p[b] = (uint8_t)(dw[b >> 2] >> (8 * (b & 3)));
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#if S3DG_KS_TRACE
    if (l == 0 && g_ks_trace) {
        // bits 48-63: HW_ID's wave/SIMD/pipe/CU/SH/SE fields (start stamp),
        // XCC_ID (end stamp); the 100 MHz clock below (tools/ks_xcd_lab.py)
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const uint64_t wi = bid * W + w, m48 = (1ull << 48) - 1;
        g_ks_trace[2 * wi] = (t_start & m48) | ((uint64_t)(hw & 0xFFFFu) << 48);
        g_ks_trace[2 * wi + 1] = (wall_clock64() & m48) | ((uint64_t)(xcc & 0xFu) << 48);
    }
#endif
}

// Persistent launches: the next work unit for a wave on XCD x.  Queue v holds
// the wave units of the static grid's workgroups b = v (mod 8) in order
// (q -> workgroup 8*(q/W) + v, wave q%W): the units XCD v would have been dealt.
// A wave drains its own XCD's queue, then takes from the others', so an XCD
// that runs ahead takes over the work of a slower one instead of idling at the
// end of the launch.  One device-scope fetch-add (lane 0, vector memory) per
// attempt; `gone` marks the queues found empty (wave-uniform).
template <int W>
__device__ __forceinline__ bool ks_take(const KeystreamArgs &A, const KeystreamArgs &A2, uint64_t *ctr, uint32_t x,
                                        uint32_t l, uint32_t &gone, uint64_t &b, uint32_t &w, bool &second) {
    for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t v = (x + i) & 7;
        if (gone & (1u << v)) continue;
        const uint64_t quota = (uint64_t)W * ((A.nwg + 7 - v) / 8);
        const uint64_t quota2 = (uint64_t)W * ((A2.nwg + 7 - v) / 8);   // A2.nwg = 0: no second set
        uint64_t q = 0;
        if (l == 0) q = __hip_atomic_fetch_add(ctr + 16 * v, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        q = readlane64(q, 0);
        if (q < quota) {
            b = 8 * (q / W) + v;
            w = (uint32_t)(q % W);
            second = false;
            return true;
        }
        if (q - quota < quota2) {
            q -= quota;
            b = 8 * (q / W) + v;
            w = (uint32_t)(q % W);
            second = true;
            return true;
        }
        gone |= 1u << v;
    }
    return false;
}

// Keystream launch.  Static grid (A.ctr null): workgroup blockIdx.x does its
// own W units.  Persistent (A.ctr set, launches of more than one round of
// resident waves): gridDim.x workgroups stay resident and every wave takes
// units from the per-XCD queues until all are empty; counter set A.par of
// A.ctr serves this launch, and workgroup 0 zeroes the other set for the next
// launch on the stream (launches on one stream never overlap).  Each queue
// holds its XCD's units of A, then its units of A2 (A2.nwg > 0: the launch's
// last chunks with shorter lanes, so the launch drains on shorter units).
template <int D, int W, int SP>
__global__ __launch_bounds__(64 * W) void k_keystream(uint8_t *dst, KeystreamArgs A, const uint64_t *jtab,
                                                      KeystreamArgs A2, const uint64_t *jtab2) {
    constexpr int RS = D * 8 + 16;
    __shared__ __attribute__((aligned(16))) uint8_t rows[W][64 * RS];
    const uint32_t t = threadIdx.x, l = t & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
    uint8_t *myrows = rows[w];
    if (!A.ctr) {
        ks_unit<D, W, SP>(dst, A, jtab, myrows, l, ks_remap(A, blockIdx.x), w);
        return;
    }
    uint64_t *const cur = A.ctr + (A.par ? 128 : 0);   // 8 counters, 128 B apart
    if (blockIdx.x == 0 && t < 8)
        __hip_atomic_store(A.ctr + (A.par ? 0 : 128) + 16 * t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t x = blockIdx.x & 7;
    uint32_t gone = 0, ww = 0;
    uint64_t b = 0;
    bool second = false;
    while (ks_take<W>(A, A2, cur, x, l, gone, b, ww, second)) {
        if (second) ks_unit<D, W, SP>(dst, A2, jtab2, myrows, l, ks_remap(A2, b), ww);
        else ks_unit<D, W, SP>(dst, A, jtab, myrows, l, ks_remap(A, b), ww);
    }
}

// DG1 zero prefixes in the fill's store shape (paired with a keystream launch
// over the chunks' tails, s3dg_internal_dgen_chunk): one 64-thread workgroup
// per 4 KiB granule, four 16-byte zero stores per lane (1 KiB per
// instruction).  2D grid: x = granule of the chunk, padded to zgp (a multiple
// of 8), y = chunk, so the linear workgroup id y*zgp + x, dealt round-robin
// to the XCDs, lands on XCD x mod 8 and writes granule x of its chunk, = x
// (mod 8) in the buffer: every XCD on every 8th granule, as the fill
// (DESIGN.md §5.1).  The dgen keystream's own all-zero waves write 64 lane
// regions per wave instead (§5.2).  Chunk y -> object y / cpo by Lemire's
// fastdiv (m_cpo = floor(2^64 / cpo) + 1; y, cpo < 2^32).  That constant wraps
// to 0 for cpo == 1 (one chunk per object, e.g. a ragged [0,1) block range), so
// that case takes ko = y directly (a uniform branch).
template <int SP, int NW>
__global__ __launch_bounds__(64 * NW) void k_zero_prefix(uint8_t *dst, uint64_t y0, uint64_t cpo, uint64_t m_cpo,
                                                         uint64_t obj_stride, uint64_t chunk_bytes, uint32_t zw) {
    const uint32_t x = blockIdx.x;
    if ((uint64_t)x * kBlk >= zw) return;
    const uint32_t lim = zw - x * kBlk;   // bytes of this granule below zw (a multiple of 16)
    const uint64_t y = y0 + blockIdx.y;
    const uint64_t ko = cpo == 1 ? y : __umul64hi(m_cpo, y);
    const uint64_t cl = y - ko * cpo;
    uint64_t off = ko * obj_stride + cl * chunk_bytes + (uint64_t)x * kBlk;
    asm volatile("" : "+v"(off));   // the address on the VALU
    uint8_t *p = dst + off + threadIdx.x * 16;
    const u32x4 z = {0u, 0u, 0u, 0u};
    if (lim >= kBlk) {
#pragma unroll
        for (int k = 0; k < 4 / NW; ++k) store16<SP>(p + k * 1024 * NW, z);
    } else {   // the partial last granule
#pragma unroll
        for (int k = 0; k < 4 / NW; ++k)
            if (threadIdx.x * 16 + k * 1024 * NW < lim) store16<SP>(p + k * 1024 * NW, z);
    }
}

template <int SP, int NW>
void launch_zp_one(dim3 g, uint32_t lds, hipStream_t s, uint8_t *dst, uint64_t y0, uint64_t cpo, uint64_t m_cpo,
                   uint64_t obj_stride, uint64_t chunk_bytes, uint32_t zw) {
    hipLaunchKernelGGL((k_zero_prefix<SP, NW>), g, dim3(64 * NW), lds, s, dst, y0, cpo, m_cpo, obj_stride,
                       chunk_bytes, zw);
}

template <int D, int W>
hipError_t launch_ks_one(uint8_t *dst, const KeystreamArgs &A, const uint64_t *jtab, uint32_t lds,
                         int store, hipStream_t s, uint64_t wgs, const KeystreamArgs &A2, const uint64_t *jtab2) {
    if (wgs > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const dim3 g((uint32_t)wgs), t(64 * W);
    if (store == kStoreSC1)
        hipLaunchKernelGGL((k_keystream<D, W, kStoreSC1>), g, t, lds, s, dst, A, jtab, A2, jtab2);
    else if (store == kStoreNTSC1)
        hipLaunchKernelGGL((k_keystream<D, W, kStoreNTSC1>), g, t, lds, s, dst, A, jtab, A2, jtab2);
    else if (store == kStoreNT)
        hipLaunchKernelGGL((k_keystream<D, W, kStoreNT>), g, t, lds, s, dst, A, jtab, A2, jtab2);
    else
        hipLaunchKernelGGL((k_keystream<D, W, kStorePlain>), g, t, lds, s, dst, A, jtab, A2, jtab2);
    return hipGetLastError();
}

template <int D, int W>
hipError_t occ_ks_one(uint32_t lds, int *out) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        out, reinterpret_cast<const void *>(&k_keystream<D, W, kStorePlain>), 64 * W, lds);
}

// static LDS of k_keystream<D, W>
constexpr uint32_t ks_static_lds(int D, int W) { return (uint32_t)W * 64u * (uint32_t)(D * 8 + 16); }

#define S3DG_KS_DISPATCH(r, fn, sh, ...)                                         \
    do {                                                                         \
        const int d_ = (sh).draws, w_ = (sh).waves;                              \
        if (d_ == 64) r = (w_ == 1 ? fn<64, 1>(__VA_ARGS__) : w_ == 2 ? fn<64, 2>(__VA_ARGS__) : fn<64, 4>(__VA_ARGS__)); \
        else if (d_ == 32) r = (w_ == 1 ? fn<32, 1>(__VA_ARGS__) : w_ == 2 ? fn<32, 2>(__VA_ARGS__) : fn<32, 4>(__VA_ARGS__)); \
        else r = (w_ == 1 ? fn<16, 1>(__VA_ARGS__) : w_ == 2 ? fn<16, 2>(__VA_ARGS__) : fn<16, 4>(__VA_ARGS__)); \
    } while (0)

// Grid sizes are 32-bit WORK-ITEM counts in the AQL dispatch packet: cap a
// launch at 2^22 workgroups per dimension (x 256 threads < 2^32).
constexpr uint64_t kMaxGridX = 1ull << 22;
// Batch launches (k_fill_batch, 64 x NW threads): the largest multiple of 256
// workgroups (XCD dealing and the prefetch spans restart at each launch) whose
// work items still fit in 32 bits, so a config-2 step (20.5 M blocks) is one
// launch instead of five.  Env S3DG_BATCH_GRID_CAP (a multiple of 256)
// overrides it, for A/Bs and for the tests of the split path.
uint64_t batch_grid_cap(int nw) {
#ifdef S3DG_DIAG_GRID_CAP
    (void)nw;
    return S3DG_DIAG_GRID_CAP;   // diagnostic builds (tools/variant_lab.py A/B)
#endif
    static const uint64_t env = [] {
        const char *v = getenv("S3DG_BATCH_GRID_CAP");
        const uint64_t x = v ? strtoull(v, nullptr, 10) : 0;
        return x >= 256 ? x & ~255ull : 0ull;
    }();
    const uint64_t lim = (0xFFFFFFFFull / (64ull * (uint64_t)nw)) & ~255ull;
    return env && env < lim ? env : lim;
}

template <int NT, int NW>
void launch_stream_one(dim3 g, uint32_t lds, hipStream_t s, uint8_t *d, const u32x4 *b, uint64_t stride,
                       uint64_t ent0, uint64_t obj_size, uint32_t blk_lo, PrefixParams pp) {
    hipLaunchKernelGGL((k_fill_stream<NT, NW>), g, dim3(64 * NW), lds, s, d, b, stride, ent0, obj_size, blk_lo, pp);
}

template <int NT, int NW>
void launch_batch_one(dim3 g, uint32_t lds, hipStream_t s, uint8_t *d, const TileRec *tiles,
                      uint64_t ntiles, uint64_t g0, uint32_t pf, uint32_t tshift, const u32x4 *b, uint32_t rt_floor) {
    if (rt_floor)
        hipLaunchKernelGGL((k_fill_batch<NT, NW, false, true>), g, dim3(64 * NW), lds, s, d, tiles, ntiles, g0, pf,
                           tshift, b, rt_floor);
    else
        hipLaunchKernelGGL((k_fill_batch<NT, NW>), g, dim3(64 * NW), lds, s, d, tiles, ntiles, g0, pf, tshift, b,
                           0u);
}

template <int NT, int NW>
void launch_batch_abl_one(dim3 g, uint32_t lds, hipStream_t s, uint8_t *d, const TileRec *tiles,
                          uint64_t ntiles, uint64_t g0, uint32_t pf, uint32_t tshift, const u32x4 *b, uint32_t pace) {
    hipLaunchKernelGGL((k_fill_batch<NT, NW, true>), g, dim3(64 * NW), lds, s, d, tiles, ntiles, g0, pf, tshift, b,
                       pace);
}

template <int NT, int NW>
void launch_ceiling_one(dim3 g, uint32_t lds, hipStream_t s, uint8_t *d, uint64_t nch, uint64_t g0,
                        uint32_t pattern, const TileRec *thr, uint64_t nthr, uint32_t pf) {
    hipLaunchKernelGGL((k_write_ceiling<NT, NW>), g, dim3(64 * NW), lds, s, d, nch, g0, pattern, thr, nthr, pf);
}

#define S3DG_DISPATCH_W(SP, fn, lc, ...)                                        \
    do {                                                                        \
        if (lc.waves_per_block == 1) fn<SP, 1>(__VA_ARGS__);                    \
        else if (lc.waves_per_block == 4) fn<SP, 4>(__VA_ARGS__);               \
        else fn<SP, 2>(__VA_ARGS__);                                            \
    } while (0)
#define S3DG_DISPATCH(fn, lc, ...)                                              \
    do {                                                                        \
        if (lc.store == kStoreNT) S3DG_DISPATCH_W(kStoreNT, fn, lc, __VA_ARGS__);    \
        else if (lc.store == kStoreSC1) S3DG_DISPATCH_W(kStoreSC1, fn, lc, __VA_ARGS__); \
        else if (lc.store == kStoreNTSC1) S3DG_DISPATCH_W(kStoreNTSC1, fn, lc, __VA_ARGS__); \
        else S3DG_DISPATCH_W(kStorePlain, fn, lc, __VA_ARGS__);                \
    } while (0)

template <int NT, int NW>
hipError_t occ_one(bool batch, uint32_t lds, int *out) {
    if (batch)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            out, reinterpret_cast<const void *>(&k_fill_batch<NT, NW>), 64 * NW, lds);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        out, reinterpret_cast<const void *>(&k_fill_stream<NT, NW>), 64 * NW, lds);
}

}  // namespace

#define S3DG_DISPATCH_RET_W(r, SP, fn, lc, ...)                                 \
    do {                                                                        \
        if (lc.waves_per_block == 1) r = fn<SP, 1>(__VA_ARGS__);                \
        else if (lc.waves_per_block == 4) r = fn<SP, 4>(__VA_ARGS__);           \
        else r = fn<SP, 2>(__VA_ARGS__);                                        \
    } while (0)
#define S3DG_DISPATCH_RET(r, fn, lc, ...)                                       \
    do {                                                                        \
        if (lc.store == kStoreNT) S3DG_DISPATCH_RET_W(r, kStoreNT, fn, lc, __VA_ARGS__);    \
        else if (lc.store == kStoreSC1) S3DG_DISPATCH_RET_W(r, kStoreSC1, fn, lc, __VA_ARGS__); \
        else if (lc.store == kStoreNTSC1) S3DG_DISPATCH_RET_W(r, kStoreNTSC1, fn, lc, __VA_ARGS__); \
        else S3DG_DISPATCH_RET_W(r, kStorePlain, fn, lc, __VA_ARGS__);         \
    } while (0)

uint32_t occupancy_lds(int wgs, uint32_t static_lds) {
    if (wgs <= 0) return 0;
    constexpr uint32_t kLdsPerCu = 160u * 1024u, kGranule = 512u;
    // smallest granule-rounded footprint with floor(kLdsPerCu / footprint) == wgs
    uint32_t total = (kLdsPerCu / (uint32_t)(wgs + 1)) / kGranule * kGranule + kGranule;
    if (total < static_lds) return 0;
    return total - static_lds;
}

hipError_t fill_occupancy(const LaunchCfg &lc, bool batch, int *wgs_per_cu) {
    hipError_t e;
    S3DG_DISPATCH_RET(e, occ_one, lc, batch, lc.dyn_lds, wgs_per_cu);
    return e;
}

hipError_t launch_fill_stream(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size,
                              uint64_t stride, uint64_t n_objs, uint32_t blk_lo,
                              uint32_t blk_hi, uint64_t seed_base, uint64_t first_obj,
                              PrefixParams pp, const void *base_dev, hipStream_t s) {
    (void)hipGetLastError();   // drop stale errors of unrelated calls (e.g. torch pointer probes)
    const u32x4 *b = reinterpret_cast<const u32x4 *>(base_dev);
    const uint32_t nx = blk_hi - blk_lo;
    for (uint64_t y0 = 0; y0 < n_objs; y0 += 65535) {
        const uint32_t ny = (uint32_t)((n_objs - y0) < 65535 ? (n_objs - y0) : 65535);
        for (uint64_t x0 = 0; x0 < nx; x0 += kMaxGridX) {
            const uint32_t gx = (uint32_t)((nx - x0) < kMaxGridX ? (nx - x0) : kMaxGridX);
            S3DG_DISPATCH(launch_stream_one, lc, dim3(gx, ny), lc.dyn_lds, s, dst + y0 * stride + x0 * kBlk, b,
                          stride, seed_base + ((first_obj + y0) << 32), obj_size, (uint32_t)(blk_lo + x0), pp);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

static hipError_t batch_tiles(const LaunchCfg &lc, uint8_t *dst_base, uint64_t total_tiles, uint32_t tshift,
                              TileRec *tiles, const void *base_dev, hipStream_t s, bool ablated) {
    hipError_t e;
    const u32x4 *b = reinterpret_cast<const u32x4 *>(base_dev);
    const uint64_t total = total_tiles << tshift;
    const uint64_t cap = batch_grid_cap(lc.waves_per_block);
    for (uint64_t g0 = 0; g0 < total; g0 += cap) {
        const uint32_t gx = (uint32_t)((total - g0) < cap ? (total - g0) : cap);
        if (ablated)
            S3DG_DISPATCH(launch_batch_abl_one, lc, dim3(gx), lc.dyn_lds, s, dst_base, tiles, total_tiles, g0,
                          lc.prefetch_tiles, tshift, b, lc.pace);
        else
            S3DG_DISPATCH(launch_batch_one, lc, dim3(gx), lc.dyn_lds, s, dst_base, tiles, total_tiles, g0,
                          lc.prefetch_tiles, tshift, b, lc.rt_floor);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_batch_tiles(const LaunchCfg &lc, uint8_t *dst_base, uint64_t total_tiles, uint32_t tshift,
                              TileRec *tiles, const void *base_dev, hipStream_t s) {
    (void)hipGetLastError();
    return batch_tiles(lc, dst_base, total_tiles, tshift, tiles, base_dev, s, false);
}

hipError_t launch_batch_map(const s3dg_obj_desc *d, uint64_t n, const uint64_t *rec_lo, TileRec *tiles,
                            uint32_t tshift, uintptr_t base, uint64_t lead0, uint64_t first_off, hipStream_t s) {
    (void)hipGetLastError();
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_batch_map, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d, n, rec_lo, tiles, tshift,
                       (uint64_t)base, lead0, first_off);
    return hipGetLastError();
}

hipError_t launch_fill_uniform_tiles(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size, uint64_t stride,
                                     uint64_t n_objs, uint32_t tiles_per_obj, uint32_t tshift, uint32_t lead,
                                     uint64_t ent0, PrefixParams pp, TileRec *tiles, const void *base_dev,
                                     hipStream_t s) {
    (void)hipGetLastError();
    const uint64_t total_tiles = n_objs * tiles_per_obj;
    hipLaunchKernelGGL(k_tile_map_uniform, dim3((uint32_t)((total_tiles + 255) / 256)), dim3(256), 0, s, tiles,
                       total_tiles, tiles_per_obj, tshift, stride, obj_size, ent0, lead, pp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return batch_tiles(lc, dst, total_tiles, tshift, tiles, base_dev, s, false);
}

// The write ceiling in the tiled fill's own shape: the same records, grid,
// LDS image, barrier, stores and trailing prefetch as a uniform stream
// through k_fill_batch, without the PRNG chain and the window patches.
hipError_t launch_fill_uniform_tiles_ablated(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size, uint64_t stride,
                                             uint64_t n_objs, uint32_t tiles_per_obj, uint32_t tshift, uint32_t lead,
                                             PrefixParams pp, TileRec *tiles, const void *base_dev, hipStream_t s) {
    (void)hipGetLastError();
    const uint64_t total_tiles = n_objs * tiles_per_obj;
    hipLaunchKernelGGL(k_tile_map_uniform, dim3((uint32_t)((total_tiles + 255) / 256)), dim3(256), 0, s, tiles,
                       total_tiles, tiles_per_obj, tshift, stride, obj_size, 0ull, lead, pp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return batch_tiles(lc, dst, total_tiles, tshift, tiles, base_dev, s, true);
}

// Persistent keystream launches from this many rounds of resident waves up.
// Whole libraries in one process, interleaved: persistent
// for any launch of more than one round against the static grid
// (profiles/r04/k/pass1/lib_ab.log): one 80 GiB DG1 launch 6715 -> 7011 GB/s,
// K2 84 GB in one launch 6763 -> 7087, ten 8 GiB DG1 launches (8 rounds each)
// 6248 -> 6441, but K2 8 GiB launches (4 rounds of 4096-draw lanes)
// 6417 -> 6388 and DG1 with a zero prefix (4-wave workgroups, short
// all-zero units) 6204 -> 6018.  From 6 rounds, 1-wave workgroups only
// (profiles/r04/k/lib_ab.log): the three gains kept (6421 / 6987 / 7052
// against 6232 / 6646 / 6705), 4-round launches unchanged (persistent from
// one round: DG1 4 GiB launches 6175 -> 6151, K2 8 GiB 6400 -> 6376).
#ifndef S3DG_KS_PERSIST_ROUNDS
#define S3DG_KS_PERSIST_ROUNDS 6
#endif
constexpr uint32_t kKsPersistRounds = S3DG_KS_PERSIST_ROUNDS;

// Resident workgroups per CU of a keystream shape (cached: the occupancy
// query is a host-side calculation, but a host call's latency budget is µs).
static int ks_resident_per_cu(const KsShape &sh, uint32_t lds) {
    static std::mutex mu;
    static std::map<uint64_t, int> cache;
    const uint64_t key = ((uint64_t)sh.draws << 48) | ((uint64_t)sh.waves << 40) | lds;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    hipError_t e;
    S3DG_KS_DISPATCH(e, occ_ks_one, sh, lds, &n);
    if (e != hipSuccess) n = 0;
    (void)hipGetLastError();
    cache[key] = n;
    return n;
}

hipError_t launch_keystream(uint8_t *dst, const KeystreamArgs &A0, const uint64_t *jtab,
                           const KsShape &sh, hipStream_t s, KsCounters *ctrs, int cus, int persist_rounds,
                           const KeystreamArgs *tail, const uint64_t *tail_jtab) {
    (void)hipGetLastError();
    const uint32_t lds = occupancy_lds(sh.wgs_per_cu, ks_static_lds(sh.draws, sh.waves));
    const uint32_t xg = sh.xcd_waves > sh.waves ? (uint32_t)(sh.xcd_waves / sh.waves) : 1u;
    // static-grid workgroups of an argument set
    auto grid_of = [&](KeystreamArgs &X) -> uint64_t {
        X.xg = xg;
        const uint64_t waves = (X.nchunks * X.lpc + 63) / 64;
        const uint64_t wgs = (waves + sh.waves - 1) / sh.waves;
        X.nwg = (uint32_t)(wgs > 0x7FFFFFFFull ? 0x7FFFFFFFull : wgs);
        X.ctr = nullptr;
        X.par = 0;
        return wgs;
    };
    KeystreamArgs A = A0, A2{};
    const uint64_t wgs = grid_of(A);
    uint64_t wgs2 = 0;
    if (tail) {
        A2 = *tail;
        wgs2 = grid_of(A2);
    }
    if (wgs > 0x7FFFFFFFull || wgs2 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    uint64_t grid = wgs;
    bool persistent = false;
#if !S3DG_DIAG_KS_STATIC
    // at least `rounds` rounds of resident waves (default: 1-wave workgroups
    // from kKsPersistRounds): a persistent grid over per-XCD queues
    // (k_keystream), one resident round of workgroups, a multiple of 8
    const uint64_t rounds = persist_rounds < 0 ? (sh.waves == 1 ? kKsPersistRounds : 0) : (uint64_t)persist_rounds;
    if (rounds > 0 && ctrs && ctrs->dev && cus > 0) {
        const uint64_t cap = ((uint64_t)ks_resident_per_cu(sh, lds) * (uint64_t)cus) & ~7ull;
        if (cap >= 8 && wgs + wgs2 >= rounds * cap) {
            A.ctr = ctrs->dev;
            A.par = ctrs->par;
            grid = cap;
            persistent = true;
        }
    }
#endif
    hipError_t e;
    if (persistent) {   // both sets in one launch, A's units first
        S3DG_KS_DISPATCH(e, launch_ks_one, sh, dst, A, jtab, lds, sh.store, s, grid, A2, tail_jtab);
        if (e == hipSuccess) ctrs->par ^= 1u;
        return e;
    }
    KeystreamArgs none{};   // static grid: A2 unused (nwg 0); the tail set as a launch of its own
    S3DG_KS_DISPATCH(e, launch_ks_one, sh, dst, A, jtab, lds, sh.store, s, grid, none, (const uint64_t *)nullptr);
    if (e == hipSuccess && tail)
        S3DG_KS_DISPATCH(e, launch_ks_one, sh, dst, A2, tail_jtab, lds, sh.store, s, wgs2, none,
                         (const uint64_t *)nullptr);
    return e;
}

hipError_t keystream_occupancy(const KsShape &sh, int *wgs_per_cu) {
    const uint32_t lds = occupancy_lds(sh.wgs_per_cu, ks_static_lds(sh.draws, sh.waves));
    hipError_t e;
    S3DG_KS_DISPATCH(e, occ_ks_one, sh, lds, wgs_per_cu);
    return e;
}

hipError_t launch_zero_prefix(uint8_t *dst, uint64_t nchunks, uint64_t cpo, uint64_t obj_stride, uint64_t chunk_bytes,
                              uint32_t zw, const LaunchCfg &lc, hipStream_t s) {
    (void)hipGetLastError();
    if (zw == 0 || nchunks == 0) return hipSuccess;
    if (cpo == 0 || cpo > 0xFFFFFFFFull || nchunks > 0xFFFFFFFFull || (chunk_bytes & 4095u) || (zw & 15u) ||
        zw > chunk_bytes)
        return hipErrorInvalidValue;
    const uint32_t zgp = ((zw + kBlk - 1) / kBlk + 7u) & ~7u;
    const uint64_t m_cpo = ~0ull / cpo + 1;
    for (uint64_t y0 = 0; y0 < nchunks; y0 += 65535) {
        const dim3 g(zgp, (uint32_t)((nchunks - y0) < 65535 ? (nchunks - y0) : 65535));
        S3DG_DISPATCH(launch_zp_one, lc, g, lc.dyn_lds, s, dst, y0, cpo, m_cpo, obj_stride, chunk_bytes, zw);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_write_ceiling(const LaunchCfg &lc, uint8_t *dst, uint64_t len, uint32_t pattern,
                                const TileRec *thr, uint64_t nthr, hipStream_t s) {
    (void)hipGetLastError();
    const uint64_t nch = len / kBlk;
    const uint32_t pf = thr && nthr ? lc.prefetch_tiles : 0;
    for (uint64_t g0 = 0; g0 < nch; g0 += kMaxGridX) {
        const uint32_t gx = (uint32_t)((nch - g0) < kMaxGridX ? (nch - g0) : kMaxGridX);
        S3DG_DISPATCH(launch_ceiling_one, lc, dim3(gx), lc.dyn_lds, s, dst, nch, g0, pattern, thr, nthr, pf);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace s3dg

#if S3DG_KS_TRACE
extern "C" int s3dg_diag_ks_trace(void *buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_ks_trace), &buf, sizeof(buf));
}
#endif
