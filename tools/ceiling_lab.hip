// ceiling_lab.hip — write-pattern microbenchmarks (tooling, not product).
// Which store pattern reaches the MI355X HBM write ceiling?
//   V1 persistent grid-stride, 16 B/lane per iteration (the product's ceiling kernel)
//   V2 non-persistent: workgroup b writes one contiguous chunk of `chunk` bytes
//   V3 persistent, each wave writes 4 KiB contiguous per iteration, block-interleaved
//      across waves (the sliding-window layout proposed for the fill kernel)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (u32x4 *)p);
    else *(u32x4 *)p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void v2_chunk(uint8_t *dst, uint64_t chunk, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    uint8_t *b = dst + (uint64_t)blockIdx.x * chunk;
    for (uint64_t o = threadIdx.x * 16ull; o < chunk; o += 256 * 16) st<NT>(b + o, v);
}

template <bool NT>
__global__ __launch_bounds__(256) void v3_blocks(uint8_t *dst, uint64_t nblk, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * 4;
    for (uint64_t g = w; g < nblk; g += W) {
        uint8_t *b = dst + g * 4096;
#pragma unroll
        for (int j = 0; j < 4; ++j) st<NT>(b + j * 1024 + lane * 16, v);
    }
}

extern "C" {
__attribute__((visibility("default"))) int lab_v2(void *dst, uint64_t len, uint64_t chunk, int nt, void *s) {
    dim3 g((unsigned)(len / chunk));
    if (nt) hipLaunchKernelGGL(v2_chunk<true>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u);
    else hipLaunchKernelGGL(v2_chunk<false>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u);
    return (int)hipGetLastError();
}
__attribute__((visibility("default"))) int lab_v3(void *dst, uint64_t len, int grid, int nt, void *s) {
    if (nt) hipLaunchKernelGGL(v3_blocks<true>, dim3(grid), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, len / 4096, 7u);
    else hipLaunchKernelGGL(v3_blocks<false>, dim3(grid), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, len / 4096, 7u);
    return (int)hipGetLastError();
}
}

// ---- V4: generic (threads per WG T, bytes per WG C), non-persistent -------------
template <int T>
__global__ __launch_bounds__(T) void v4_tc(uint8_t *dst, uint64_t chunk, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    uint8_t *b = dst + (uint64_t)blockIdx.x * chunk;
    for (uint64_t o = threadIdx.x * 16ull; o < chunk; o += T * 16) st<false>(b + o, v);
}

// ---- V5: one wave per 4 KiB block, the block's PRNG computed by the wave -----------
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
__device__ __forceinline__ uint64_t sm(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void v5_wave_block(uint8_t *dst, uint64_t seed, const u32x4 *base) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t blk = (uint64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32x4 B[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) B[j] = base[j * 64 + lane];
    uint64_t x = seed + blk;
    uint64_t s0 = sm(x + 0x9E3779B97F4A7C15ull), s1 = sm(x + 2 * 0x9E3779B97F4A7C15ull);
    uint64_t s2 = sm(x + 3 * 0x9E3779B97F4A7C15ull), s3 = sm(x + 4 * 0x9E3779B97F4A7C15ull);
    uint64_t r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        r[q] = rotl64(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl64(s3, 45);
    }
    uint8_t *b = dst + blk * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        u32x4 v = B[j];
        if (j == 0 && lane < 2) { v = u32x4{(uint32_t)r[2*lane], (uint32_t)(r[2*lane] >> 32), (uint32_t)r[2*lane+1], (uint32_t)(r[2*lane+1] >> 32)}; }
        if (j == 2 && lane < 2) { v = u32x4{(uint32_t)r[4+2*lane], (uint32_t)(r[4+2*lane] >> 32), (uint32_t)r[5+2*lane], (uint32_t)(r[5+2*lane] >> 32)}; }
        st<false>(b + j * 1024 + lane * 16, v);
    }
}

extern "C" {
__attribute__((visibility("default"))) int lab_v4(void *dst, uint64_t len, uint64_t chunk, int T, void *s) {
    dim3 g((unsigned)(len / chunk));
    switch (T) {
    case 64: hipLaunchKernelGGL(v4_tc<64>, g, dim3(64), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u); break;
    case 256: hipLaunchKernelGGL(v4_tc<256>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u); break;
    case 512: hipLaunchKernelGGL(v4_tc<512>, g, dim3(512), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u); break;
    default: hipLaunchKernelGGL(v4_tc<1024>, g, dim3(1024), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u); break;
    }
    return (int)hipGetLastError();
}
__attribute__((visibility("default"))) int lab_v5(void *dst, uint64_t len, int wpb, void *base, void *s) {
    const uint64_t nb = len / 4096;
    switch (wpb) {
    case 1: hipLaunchKernelGGL(v5_wave_block<1>, dim3(nb), dim3(64), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    case 2: hipLaunchKernelGGL(v5_wave_block<2>, dim3(nb / 2), dim3(128), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    case 4: hipLaunchKernelGGL(v5_wave_block<4>, dim3(nb / 4), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    default: hipLaunchKernelGGL(v5_wave_block<8>, dim3(nb / 8), dim3(512), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    }
    return (int)hipGetLastError();
}
}

// ---- V6: WG of 4 waves writes ONE 4 KiB block (1 store/lane); waves whose KiB
// holds a window compute the PRNG chain.  MODE 0: uniform values (SALU),
// MODE 1: forced onto VALU.  ALLW: every wave computes (worst case).
template <int MODE, bool ALLW>
__global__ __launch_bounds__(256) void v6_wg_block(uint8_t *dst, uint64_t seed, const u32x4 *base) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t blk = blockIdx.x;
    u32x4 v = base[w * 64 + lane];
    if (ALLW || w == 0 || w == 2) {
        uint64_t x = seed + blk;
        if (MODE == 1) asm volatile("" : "+v"(x));
        uint64_t s0 = sm(x + 0x9E3779B97F4A7C15ull), s1 = sm(x + 2 * 0x9E3779B97F4A7C15ull);
        uint64_t s2 = sm(x + 3 * 0x9E3779B97F4A7C15ull), s3 = sm(x + 4 * 0x9E3779B97F4A7C15ull);
        uint64_t r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            r[q] = rotl64(s0 + s3, 23) + s0;
            const uint64_t t = s1 << 17;
            s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl64(s3, 45);
        }
        const int o = (w == 2) ? 4 : 0;
        if (lane < 2) {
            const uint64_t a = lane ? r[o + 2] : r[o], b = lane ? r[o + 3] : r[o + 1];
            v = u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
        }
    }
    st<false>(dst + blk * 4096 + w * 1024 + lane * 16, v);
}

extern "C" __attribute__((visibility("default"))) int lab_v6(void *dst, uint64_t len, int mode, void *base, void *s) {
    const uint64_t nb = len / 4096;
    switch (mode) {
    case 0: hipLaunchKernelGGL((v6_wg_block<0, false>), dim3(nb), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    case 1: hipLaunchKernelGGL((v6_wg_block<1, false>), dim3(nb), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    case 2: hipLaunchKernelGGL((v6_wg_block<0, true>), dim3(nb), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    default: hipLaunchKernelGGL((v6_wg_block<1, true>), dim3(nb), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base); break;
    }
    return (int)hipGetLastError();
}

// ---- V8: WG of 4 waves per block, wave 0 computes the chain once, shares via LDS.
template <int T>
__global__ __launch_bounds__(T) void v8_shared_chain(uint8_t *dst, uint64_t seed, const u32x4 *base) {
    __shared__ uint64_t R[8];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t blk = blockIdx.x;
    constexpr int NW = T / 64, SPL = 4 / NW;   // stores per lane
    if (w == 0) {
        uint64_t x = seed + blk;
        uint64_t s0 = sm(x + 0x9E3779B97F4A7C15ull), s1 = sm(x + 2 * 0x9E3779B97F4A7C15ull);
        uint64_t s2 = sm(x + 3 * 0x9E3779B97F4A7C15ull), s3 = sm(x + 4 * 0x9E3779B97F4A7C15ull);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t r = rotl64(s0 + s3, 23) + s0;
            const uint64_t t = s1 << 17;
            s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl64(s3, 45);
            if (lane == 0) R[q] = r;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
        const int seg = (w * SPL + k);              // KiB index 0..3
        u32x4 v = base[seg * 64 + lane];
        if ((seg == 0 || seg == 2) && lane < 2) {
            const int o = (seg == 2 ? 4 : 0) + 2 * lane;
            v = u32x4{(uint32_t)R[o], (uint32_t)(R[o] >> 32), (uint32_t)R[o + 1], (uint32_t)(R[o + 1] >> 32)};
        }
        st<false>(dst + blk * 4096 + seg * 1024 + lane * 16, v);
    }
}

extern "C" __attribute__((visibility("default"))) int lab_v8(void *dst, uint64_t len, int T, void *base, void *s) {
    const uint64_t nb = len / 4096;
    if (T == 256) hipLaunchKernelGGL(v8_shared_chain<256>, dim3(nb), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base);
    else if (T == 128) hipLaunchKernelGGL(v8_shared_chain<128>, dim3(nb), dim3(128), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base);
    else hipLaunchKernelGGL(v8_shared_chain<64>, dim3(nb), dim3(64), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base);
    return (int)hipGetLastError();
}
extern "C" __attribute__((visibility("default"))) int lab_v4b(void *dst, uint64_t len, uint64_t chunk, void *s) {
    hipLaunchKernelGGL(v4_tc<128>, dim3(len / chunk), dim3(128), 0, (hipStream_t)s, (uint8_t *)dst, chunk, 7u);
    return (int)hipGetLastError();
}

// ---- V9: V8 body (T=256) launched as a 2D grid (x = block in object, y = object)
__global__ __launch_bounds__(256) void v9_shared_chain_2d(uint8_t *dst, uint64_t seed, const u32x4 *base) {
    __shared__ uint64_t R[8];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t blk = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (w == 0) {
        uint64_t x = seed + blk;
        uint64_t s0 = sm(x + 0x9E3779B97F4A7C15ull), s1 = sm(x + 2 * 0x9E3779B97F4A7C15ull);
        uint64_t s2 = sm(x + 3 * 0x9E3779B97F4A7C15ull), s3 = sm(x + 4 * 0x9E3779B97F4A7C15ull);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t r = rotl64(s0 + s3, 23) + s0;
            const uint64_t t = s1 << 17;
            s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl64(s3, 45);
            if (lane == 0) R[q] = r;
        }
    }
    __syncthreads();
    const int seg = w;
    u32x4 v = base[seg * 64 + lane];
    if ((seg == 0 || seg == 2) && lane < 2) {
        const int o = (seg == 2 ? 4 : 0) + 2 * lane;
        v = u32x4{(uint32_t)R[o], (uint32_t)(R[o] >> 32), (uint32_t)R[o + 1], (uint32_t)(R[o + 1] >> 32)};
    }
    st<false>(dst + blk * 4096 + seg * 1024 + lane * 16, v);
}
__global__ __launch_bounds__(256) void v10_ceiling_2d(uint8_t *dst, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    const uint64_t blk = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
    st<false>(dst + blk * 4096 + threadIdx.x * 16, v);
}
extern "C" __attribute__((visibility("default"))) int lab_v9(void *dst, uint64_t len, int nx, int which, void *base, void *s) {
    const uint64_t nb = len / 4096;
    if (which == 0) hipLaunchKernelGGL(v9_shared_chain_2d, dim3(nx, nb / nx), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 5ull, (const u32x4 *)base);
    else hipLaunchKernelGGL(v10_ceiling_2d, dim3(nx, nb / nx), dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, 7u);
    return (int)hipGetLastError();
}

// V11: K2's store shape without the PRNG.  Each wave owns a chunk of 64 lane
// regions of R bytes; iteration `it` writes `seg` bytes at offset it*seg of
// every region, as seg/16 store instructions of (1024/seg) rows x seg bytes.
// V12: each wave writes its 64*R chunk front to back, 1 KiB per instruction.
template <int SEG, bool NT = false>
__global__ __launch_bounds__(256) void v11_strided(uint8_t *dst, uint64_t nchunks, uint32_t R, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    const uint32_t l = threadIdx.x & 63;
    const uint64_t wv = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wv >= nchunks) return;
    uint8_t *c = dst + wv * 64ull * R;
    constexpr uint32_t lpr = SEG / 16, rpi = 1024 / SEG;
    for (uint32_t it = 0; it < R / SEG; ++it)
#pragma unroll
        for (uint32_t i = 0; i < lpr; ++i) {
            const uint32_t row = i * rpi + l / lpr;
            st<NT>(c + (uint64_t)row * R + it * SEG + (l % lpr) * 16, v);
        }
}
__global__ __launch_bounds__(256) void v12_wave_seq(uint8_t *dst, uint64_t nchunks, uint32_t R, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    const uint32_t l = threadIdx.x & 63;
    const uint64_t wv = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wv >= nchunks) return;
    uint8_t *c = dst + wv * 64ull * R;
    for (uint64_t o = 0; o < 64ull * R; o += 1024) st<false>(c + o + l * 16, v);
}
extern "C" __attribute__((visibility("default"))) int lab_v11(void *dst, uint64_t len, uint32_t R, int seg, void *s) {
    const uint64_t nch = len / (64ull * R);
    const dim3 g((uint32_t)((nch + 3) / 4));
    switch (seg) {
    case 64: hipLaunchKernelGGL(v11_strided<64>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    case 128: hipLaunchKernelGGL(v11_strided<128>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    case 256: hipLaunchKernelGGL(v11_strided<256>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    case 512: hipLaunchKernelGGL(v11_strided<512>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    case 1024: hipLaunchKernelGGL(v11_strided<1024>, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    default: hipLaunchKernelGGL(v12_wave_seq, g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u); break;
    }
    return (int)hipGetLastError();
}

// V11 variants: nontemporal stores; occupancy forced down by dynamic LDS (lds_bytes per WG)
extern "C" __attribute__((visibility("default"))) int lab_v11x(void *dst, uint64_t len, uint32_t R, int seg, int nt,
                                                               uint32_t lds_bytes, void *s) {
    const uint64_t nch = len / (64ull * R);
    const dim3 g((uint32_t)((nch + 3) / 4));
    if (nt) {
        if (seg == 128) hipLaunchKernelGGL((v11_strided<128, true>), g, dim3(256), lds_bytes, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u);
        else hipLaunchKernelGGL((v11_strided<512, true>), g, dim3(256), lds_bytes, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u);
    } else {
        if (seg == 128) hipLaunchKernelGGL((v11_strided<128, false>), g, dim3(256), lds_bytes, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u);
        else hipLaunchKernelGGL((v11_strided<512, false>), g, dim3(256), lds_bytes, (hipStream_t)s, (uint8_t *)dst, nch, R, 7u);
    }
    return (int)hipGetLastError();
}

// V13: K2's store shape with XCD-aware region ownership.  Regions are `R`
// bytes; workgroups are dealt round-robin to the 8 XCDs, so workgroup b
// (XCD b mod 8) takes regions = b (mod 8) only: region (b>>3)*256*8 + 8*lw + (b&7)
// for its 256 lanes lw.  Each lane writes its region in `seg`-byte stages, rows
// as K2 (seg/16 lanes per row).  xcd=0: the same stages, wave-contiguous regions (V11).
// Policy: 0 plain, 2 sc1, 3 nt sc1.
template <int POL>
__device__ __forceinline__ void stp(uint8_t *p, u32x4 v) {
    if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else *(u32x4 *)p = v;
}
template <int SEG, int POL>
__global__ __launch_bounds__(256) void v13_xcd(uint8_t *dst, uint64_t nreg, uint32_t R, int xcd, uint32_t pat) {
    const u32x4 v = {pat, pat + 1, pat + 2, pat + 3};
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t b = blockIdx.x;
    constexpr uint32_t lpr = SEG / 16, rpi = 64 / lpr;
    // region of row `row` of this wave
    auto region = [&](uint32_t row) -> uint64_t {
        const uint32_t lw = w * 64 + row;
        return xcd ? (b >> 3) * 2048 + 8ull * lw + (b & 7) : b * 256 + lw;
    };
    for (uint32_t it = 0; it < R / SEG; ++it)
#pragma unroll
        for (uint32_t i = 0; i < lpr; ++i) {
            const uint32_t row = i * rpi + l / lpr;
            const uint64_t rg = region(row);
            if (rg < nreg) stp<POL>(dst + rg * R + it * SEG + (l % lpr) * 16, v);
        }
}
extern "C" __attribute__((visibility("default"))) int lab_v13(void *dst, uint64_t len, uint32_t R, int seg, int xcd,
                                                              int pol, void *s) {
    const uint64_t nreg = len / R;
    const dim3 g((uint32_t)((nreg + 2047) / 2048 * 8));
#define V13(SG, P) hipLaunchKernelGGL((v13_xcd<SG, P>), g, dim3(256), 0, (hipStream_t)s, (uint8_t *)dst, nreg, R, xcd, 7u)
    if (seg == 512 && pol == 0) V13(512, 0);
    else if (seg == 512 && pol == 2) V13(512, 2);
    else if (seg == 512 && pol == 3) V13(512, 3);
    else if (seg == 1024 && pol == 2) V13(1024, 2);
    else if (seg == 256 && pol == 2) V13(256, 2);
    else return -1;
#undef V13
    return (int)hipGetLastError();
}
