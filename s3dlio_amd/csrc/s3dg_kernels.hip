// s3dg_kernels.hip — CDNA4 (gfx950) kernels for s3dlio's synthetic payload
// generator.  Semantics: /root/reference/src/data_gen.rs:151-224
// (fill_controlled_data), bit-exact for a given entropy and base block.
//
// Work decomposition:
//   * A "tile" = up to 64 consecutive 4 KiB blocks of ONE object, owned by
//     one wave64.  Lane l first computes everything block (tile_first + l)
//     needs — u = i % U, the zero-prefix length, the SplitMix64 seed
//     expansion and the <= 8 Xoshiro256++ draws of its two 32-byte windows —
//     so the sequential-PRNG work is spread one block per lane.  The window
//     bytes go to a per-wave LDS image, the scalar block metadata stays in
//     VGPRs and is broadcast with v_readlane.
//   * The wave then writes its 64 blocks in order: 4 x 1 KiB
//     global_store_dwordx4 per block (16 B per lane, fully coalesced), data =
//     the base block held in 16 VGPRs per lane, or zeros.  Only the <= 6
//     lane-segments per block that straddle a window / the zero boundary /
//     the object tail take the masked slow path (LDS window read +
//     v_alignbyte).  No HBM reads: dedup blocks are recomputed, not copied.
//   * Persistent grid (CUs x wg_per_cu workgroups of 4 waves), grid-stride
//     over tiles.  Write-only streaming: there is no reuse, so the block->XCD
//     placement only matters for load balance.
#include "s3dg_internal.h"

namespace s3dg {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kImgDw = 20;   // per-block LDS window image: pad,W1[8],pad,W2[8],pad,unused

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

// Byte masks over the dword at byte position p.
__device__ __forceinline__ uint32_t keep_ge(int p, int e) {   // bytes with pos >= e
    int t = e - p;
    return t <= 0 ? 0xFFFFFFFFu : (t >= 4 ? 0u : (0xFFFFFFFFu << (8 * t)));
}
__device__ __forceinline__ uint32_t keep_lt(int p, int e) {   // bytes with pos < e
    int t = e - p;
    return t <= 0 ? 0u : (t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * t)) - 1u));
}

// Dword of a 32-byte window image starting at window-relative byte `rel`
// (clamped to [-4, 32]; bytes outside the window are masked by the caller).
__device__ __forceinline__ uint32_t window_dword(const uint32_t *img, int rel) {
    rel = rel < -4 ? -4 : (rel > 32 ? 32 : rel);
    const int idx = (rel + 4) >> 2;                 // 0..9 (img[0] is the pad)
    const uint32_t d0 = img[idx], d1 = img[idx + 1];
    return __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)(rel & 3));
}

// Full byte-exact value of the dword at block byte p (slow path).
__device__ __forceinline__ uint32_t patch_dword(uint32_t b, int p, int c, int m, int so,
                                                bool w2, const uint32_t *img) {
    uint32_t res = b & keep_ge(p, c);                          // zero prefix, :209-210
    const uint32_t m1 = keep_ge(p, c) & keep_lt(p, c + m);     // first window, :217
    res = (res & ~m1) | (window_dword(img, p - c) & m1);
    if (w2) {                                                  // second window, :218-221
        const uint32_t m2 = keep_ge(p, so) & keep_lt(p, so + m);
        res = (res & ~m2) | (window_dword(img + 9, p - so) & m2);
    }
    return res;
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    else *reinterpret_cast<u32x4 *>(p) = v;
}

struct Tile {
    uint8_t *dst;        // byte address of block `first`
    uint64_t size;       // object size in bytes
    uint64_t entropy;    // call_entropy of the object
    uint32_t first;      // first block index (within the object)
    uint32_t count;      // blocks in this tile, 1..64
    PrefixParams pp;
};

// One wave generates one tile.  `B` = this lane's 4 x 16 B of the base block
// (bytes j*1024 + lane*16 .. +16), `img` = this wave's LDS image (64 x 20 dw).
template <bool NT>
__device__ __forceinline__ void run_tile(const Tile &T, const u32x4 (&B)[4], uint32_t *img,
                                         uint32_t lane) {
    // ---- phase 1: lane-parallel per-block parameters + PRNG ----------------
    const bool valid = lane < T.count;
    const uint32_t i = T.first + lane;
    const uint32_t u = i % T.pp.unique;                                  // :201
    const uint64_t off = (uint64_t)i * kBlk;
    const uint32_t L = valid ? (uint32_t)((T.size - off) < kBlk ? (T.size - off) : kBlk) : 0u;
    uint32_t cl = T.pp.floor_len;
    if (T.pp.rem) {
        const uint64_t r = T.pp.rem, d = T.pp.f_den;
        cl += (uint32_t)(((uint64_t)(u + 1) * r) / d - ((uint64_t)u * r) / d);
    }
    const uint32_t c = cl < L ? cl : L;                                  // :209
    const uint32_t m = (L - c) < kMod ? (L - c) : kMod;                  // :212-214
    const uint32_t so = c > kHalf ? c : kHalf;                           // :218
    const bool w2 = m > 0 && so + m <= L;                                // :219

    uint64_t x = (uint64_t)u + T.entropy;                                // :202
    Xoshiro g;
    g.s0 = splitmix_next(x);
    g.s1 = splitmix_next(x);
    g.s2 = splitmix_next(x);
    g.s3 = splitmix_next(x);
    uint64_t r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = g.next();
    // fill_bytes_via_next: k1 draws per window, last one >>32 if its tail is 1..4 B.
    const uint32_t k1 = (m + 7) >> 3;
    const uint32_t tail = m & 7;
    const bool tail_hi = tail >= 1 && tail <= 4;
    uint64_t w1[4], w2w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        w1[q] = r[q];
        w2w[q] = k1 == 4 ? r[4 + q] : (k1 == 3 ? r[3 + q] : (k1 == 2 ? r[2 + q] : r[1 + q]));
        if (tail_hi && (uint32_t)q + 1 == k1) { w1[q] >>= 32; w2w[q] >>= 32; }
    }
    uint32_t *mine = img + lane * kImgDw;
    u32x4 *mv = reinterpret_cast<u32x4 *>(mine);
    mv[0] = u32x4{0u, (uint32_t)w1[0], (uint32_t)(w1[0] >> 32), (uint32_t)w1[1]};
    mv[1] = u32x4{(uint32_t)(w1[1] >> 32), (uint32_t)w1[2], (uint32_t)(w1[2] >> 32), (uint32_t)w1[3]};
    mv[2] = u32x4{(uint32_t)(w1[3] >> 32), 0u, (uint32_t)w2w[0], (uint32_t)(w2w[0] >> 32)};
    mv[3] = u32x4{(uint32_t)w2w[1], (uint32_t)(w2w[1] >> 32), (uint32_t)w2w[2], (uint32_t)(w2w[2] >> 32)};
    mv[4] = u32x4{(uint32_t)w2w[3], (uint32_t)(w2w[3] >> 32), 0u, 0u};
    const uint32_t meta0 = c | (so << 16);
    const uint32_t meta1 = L | (m << 16) | ((uint32_t)w2 << 24);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 2: the wave writes its blocks, 4 x 1 KiB stores each --------
    const u32x4 zero = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < T.count; ++k) {
        const uint32_t a0 = __builtin_amdgcn_readlane(meta0, k);
        const uint32_t a1 = __builtin_amdgcn_readlane(meta1, k);
        const int bc = (int)(a0 & 0xFFFF), bso = (int)(a0 >> 16);
        const int bL = (int)(a1 & 0xFFFF), bm = (int)((a1 >> 16) & 0xFF);
        const bool bw2 = (a1 >> 24) != 0;
        uint8_t *bd = T.dst + (uint64_t)k * kBlk;
        const uint32_t *bimg = img + k * kImgDw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int o = j * 1024 + (int)lane * 16;
            const bool need = (o < bc + bm && o + 16 > bc) ||
                              (bw2 && o < bso + bm && o + 16 > bso) ||
                              (o < bL && o + 16 > bL);
            if (!need) {
                if (o + 16 <= bL) store16<NT>(bd + o, (o + 16 <= bc) ? zero : B[j]);
            } else {
                u32x4 v;
                v.x = patch_dword(B[j].x, o + 0, bc, bm, bso, bw2, bimg);
                v.y = patch_dword(B[j].y, o + 4, bc, bm, bso, bw2, bimg);
                v.z = patch_dword(B[j].z, o + 8, bc, bm, bso, bw2, bimg);
                v.w = patch_dword(B[j].w, o + 12, bc, bm, bso, bw2, bimg);
                if (o + 16 <= bL) {
                    store16<NT>(bd + o, v);
                } else {                       // ragged object tail: bytes < L only
                    const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
                    for (int b = 0; b < 16 && o + b < bL; ++b)
                        bd[o + b] = (uint8_t)(dw[b >> 2] >> (8 * (b & 3)));
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void load_base(const u32x4 *base, uint32_t lane, u32x4 (&B)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) B[j] = base[j * 64 + lane];
}

template <bool NT>
__global__ __launch_bounds__(256) void k_fill_stream(uint8_t *dst, uint64_t obj_size,
                                                     uint64_t stride, uint64_t n_objs,
                                                     uint32_t blk_lo, uint32_t blk_hi,
                                                     uint64_t seed_base, uint64_t first_obj,
                                                     PrefixParams pp, const u32x4 *base) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kWavesPerWG * 64 * kImgDw];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32x4 B[4];
    load_base(base, lane, B);
    uint32_t *img = lds + wave * 64 * kImgDw;
    const uint32_t span = blk_hi - blk_lo;
    const uint64_t tpo = (span + kTileBlocks - 1) / kTileBlocks;
    const uint64_t total = tpo * n_objs;
    const uint64_t nw = (uint64_t)gridDim.x * kWavesPerWG;
    for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerWG + wave; t < total; t += nw) {
        const uint64_t j = t / tpo;
        const uint32_t tin = (uint32_t)(t - j * tpo);
        Tile T;
        T.first = blk_lo + tin * kTileBlocks;
        T.count = (blk_hi - T.first) < kTileBlocks ? (blk_hi - T.first) : kTileBlocks;
        T.dst = dst + j * stride + (uint64_t)(T.first - blk_lo) * kBlk;
        T.size = obj_size;
        T.entropy = seed_base + ((first_obj + j) << 32);
        T.pp = pp;
        run_tile<NT>(T, B, img, lane);
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_fill_batch(uint8_t *dst_base, const ObjEntry *tab,
                                                    uint64_t n, uint64_t total_tiles,
                                                    const u32x4 *base) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kWavesPerWG * 64 * kImgDw];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32x4 B[4];
    load_base(base, lane, B);
    uint32_t *img = lds + wave * 64 * kImgDw;
    const uint64_t nw = (uint64_t)gridDim.x * kWavesPerWG;
    for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerWG + wave; t < total_tiles; t += nw) {
        // largest e with tab[e].tile_begin <= t (wave-uniform search)
        uint64_t lo = 0, hi = n;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (tab[mid].tile_begin <= t) lo = mid; else hi = mid;
        }
        const ObjEntry e = tab[lo];
        const uint32_t nb = (uint32_t)((e.size + kBlk - 1) / kBlk);
        Tile T;
        T.first = (uint32_t)(t - e.tile_begin) * kTileBlocks;
        T.count = (nb - T.first) < kTileBlocks ? (nb - T.first) : kTileBlocks;
        T.dst = dst_base + e.dst_off + (uint64_t)T.first * kBlk;
        T.size = e.size;
        T.entropy = e.entropy;
        T.pp = e.pp;
        run_tile<NT>(T, B, img, lane);
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write_ceiling(uint8_t *dst, uint64_t n16, uint32_t pat) {
    const u32x4 v = {pat, pat ^ 0x9E3779B9u, pat + 1u, ~pat};
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n16; q += stride)
        store16<NT>(dst + q * 16, v);
}

}  // namespace

hipError_t launch_fill_stream(const LaunchCfg &lc, uint8_t *dst, uint64_t obj_size,
                              uint64_t stride, uint64_t n_objs, uint32_t blk_lo,
                              uint32_t blk_hi, uint64_t seed_base, uint64_t first_obj,
                              PrefixParams pp, const void *base_dev, hipStream_t s) {
    const u32x4 *b = reinterpret_cast<const u32x4 *>(base_dev);
    if (lc.nontemporal)
        hipLaunchKernelGGL(k_fill_stream<true>, dim3(lc.grid), dim3(256), 0, s, dst, obj_size,
                           stride, n_objs, blk_lo, blk_hi, seed_base, first_obj, pp, b);
    else
        hipLaunchKernelGGL(k_fill_stream<false>, dim3(lc.grid), dim3(256), 0, s, dst, obj_size,
                           stride, n_objs, blk_lo, blk_hi, seed_base, first_obj, pp, b);
    return hipGetLastError();
}

hipError_t launch_fill_batch(const LaunchCfg &lc, uint8_t *dst_base, const ObjEntry *tab,
                             uint64_t n, uint64_t total_tiles, const void *base_dev,
                             hipStream_t s) {
    const u32x4 *b = reinterpret_cast<const u32x4 *>(base_dev);
    if (lc.nontemporal)
        hipLaunchKernelGGL(k_fill_batch<true>, dim3(lc.grid), dim3(256), 0, s, dst_base, tab, n,
                           total_tiles, b);
    else
        hipLaunchKernelGGL(k_fill_batch<false>, dim3(lc.grid), dim3(256), 0, s, dst_base, tab, n,
                           total_tiles, b);
    return hipGetLastError();
}

hipError_t launch_write_ceiling(const LaunchCfg &lc, uint8_t *dst, uint64_t len, uint32_t pattern,
                                hipStream_t s) {
    if (lc.nontemporal)
        hipLaunchKernelGGL(k_write_ceiling<true>, dim3(lc.grid), dim3(256), 0, s, dst, len / 16,
                           pattern);
    else
        hipLaunchKernelGGL(k_write_ceiling<false>, dim3(lc.grid), dim3(256), 0, s, dst, len / 16,
                           pattern);
    return hipGetLastError();
}

}  // namespace s3dg
