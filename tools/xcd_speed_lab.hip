// xcd_speed_lab.hip — diagnostic kernels (tools/xcd_speed_lab.py; not product
// code): is the keystream's slower half of XCDs
// slower at arithmetic or at stores?  1-wave workgroups, four per CU (the
// keystream's residency), each wave timing its own work with the 100 MHz
// wall clock and recording the XCC that ran it:
//   k_valu         Xoshiro256 state steps in registers (no memory traffic)
//   k_store_seq    whole 1 KiB per store instruction, each wave a contiguous run
//   k_store_lanes  the keystream's pattern: 64 lane regions per wave, 512-B
//                  pieces, two rows per store instruction
//   k_store_xcd    the fill's pattern: each wave's XCD on every 8th 4 KiB granule
// Stores are global_store_dwordx4 ... sc1, as the product's.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1(uint8_t *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void stamp(uint64_t *out, uint64_t t0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = t0;
        out[3 * blockIdx.x + 1] = wall_clock64();
        out[3 * blockIdx.x + 2] = xcc;
    }
}

__device__ __forceinline__ uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

__global__ __launch_bounds__(64) void k_valu(uint64_t *out, uint64_t *sink, uint32_t iters) {
    const uint64_t t0 = wall_clock64();
    uint64_t s0 = threadIdx.x + 1, s1 = blockIdx.x * 77 + 3, s2 = 0x9E3779B97F4A7C15ull, s3 = 12345;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        acc += rotl(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45);
    }
    if (acc == 0x12345) sink[blockIdx.x] = acc;   // keeps the loop
    stamp(out, t0);
}

__global__ __launch_bounds__(64) void k_store_seq(uint8_t *dst, uint64_t *out, uint64_t bpw, uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const u32x4 v = {threadIdx.x * 0x01010101u, blockIdx.x, 0x5A5A5A5Au, ~threadIdx.x};
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * bpw;
        for (uint64_t o = threadIdx.x * 16; o < bpw; o += 1024) st_sc1(base + o, v);
    }
    stamp(out, t0);
}

__global__ __launch_bounds__(64) void k_store_lanes(uint8_t *dst, uint64_t *out, uint32_t span, uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const uint32_t l = threadIdx.x, piece = l % 32;
    const u32x4 v = {l * 0x01010101u, blockIdx.x, 0xA5A5A5A5u, ~l};
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * 64ull * span;
        for (uint32_t it = 0; it < span / 512; ++it)
            for (int i = 0; i < 32; ++i) st_sc1(base + (uint64_t)(2 * i + l / 32) * span + it * 512 + piece * 16, v);
    }
    stamp(out, t0);
}

// every wave's XCD on every 8th 4 KiB granule (the fill's pattern): wave b
// (dealt to XCD b mod 8) writes 1 MiB per unit as 256 granules = b (mod 8)
__global__ __launch_bounds__(64) void k_store_xcd(uint8_t *dst, uint64_t *out, uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const u32x4 v = {threadIdx.x * 0x01010101u, blockIdx.x, 0x3C3C3C3Cu, ~threadIdx.x};
    const uint64_t r = blockIdx.x & 7, q = blockIdx.x >> 3, per_round = gridDim.x >> 3;
    for (uint32_t u = 0; u < units; ++u)
        for (uint32_t k = 0; k < 256; ++k) {
            uint8_t *g = dst + ((((uint64_t)u * per_round + q) * 256 + k) * 8 + r) * 4096;
            for (int i = 0; i < 4; ++i) st_sc1(g + threadIdx.x * 16 + 1024 * i, v);
        }
    stamp(out, t0);
}

// the lane pattern with `nap` s_sleep(1) (64 clocks each) after every 32-store burst
__global__ __launch_bounds__(64) void k_store_lanes_paced(uint8_t *dst, uint64_t *out, uint32_t span, uint32_t units,
                                                          uint32_t nap) {
    const uint64_t t0 = wall_clock64();
    const uint32_t l = threadIdx.x, piece = l % 32;
    const u32x4 v = {l * 0x01010101u, blockIdx.x, 0xA5A5A5A5u, ~l};
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * 64ull * span;
        for (uint32_t it = 0; it < span / 512; ++it) {
            for (int i = 0; i < 32; ++i) st_sc1(base + (uint64_t)(2 * i + l / 32) * span + it * 512 + piece * 16, v);
            for (uint32_t n = 0; n < nap; ++n) __builtin_amdgcn_s_sleep(1);
        }
    }
    stamp(out, t0);
}

// a narrow sliding window: at step j every wave b writes granule j*grid + b,
// so the resident waves write a window of grid x 4 KiB (4 MiB at 1024 waves)
// that sweeps the buffer, as the fill's dispatch order does
__global__ __launch_bounds__(64) void k_store_window(uint8_t *dst, uint64_t *out, uint64_t ngran, uint32_t nap) {
    const uint64_t t0 = wall_clock64();
    const u32x4 v = {threadIdx.x * 0x01010101u, blockIdx.x, 0x69696969u, ~threadIdx.x};
    for (uint64_t g = blockIdx.x; g < ngran; g += gridDim.x) {
        for (int i = 0; i < 4; ++i) st_sc1(dst + g * 4096 + threadIdx.x * 16 + 1024 * i, v);
        for (uint32_t n = 0; n < nap; ++n) __builtin_amdgcn_s_sleep(1);   // `nap` x 64 clocks per 4 KiB granule
    }
    stamp(out, t0);
}

// the lane pattern with data that changes every store (a 32-bit LCG per lane)
__global__ __launch_bounds__(64) void k_store_lanes_rnd(uint8_t *dst, uint64_t *out, uint32_t span, uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const uint32_t l = threadIdx.x, piece = l % 32;
    uint32_t x = l * 2654435761u + blockIdx.x * 40503u + 1u;
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * 64ull * span;
        for (uint32_t it = 0; it < span / 512; ++it)
            for (int i = 0; i < 32; ++i) {
                x = x * 1664525u + 1013904223u;
                const u32x4 v = {x, x ^ 0x9E3779B9u, x * 3u, ~x};
                st_sc1(base + (uint64_t)(2 * i + l / 32) * span + it * 512 + piece * 16, v);
            }
    }
    stamp(out, t0);
}

// one 4 KiB granule per workgroup over a grid of every granule (the fill's
// dispatch shape without its PRNG, LDS image and base-block loads)
__global__ __launch_bounds__(64) void k_store_granule(uint8_t *dst, uint64_t *out) {
    const uint64_t t0 = wall_clock64();
    const u32x4 v = {threadIdx.x * 0x01010101u, blockIdx.x, 0x96969696u, ~threadIdx.x};
    const uint64_t g = blockIdx.x;
    for (int i = 0; i < 4; ++i) st_sc1(dst + g * 4096 + threadIdx.x * 16 + 1024 * i, v);
    stamp(out, t0);
}

// the lane pattern with `s_waitcnt vmcnt(N)` after every 32-store burst: at
// most N stores of the wave left in flight before it goes on (a wave of the
// fill waits on its base-block loads, and so on its earlier stores, each block)
template <int N>
__global__ __launch_bounds__(64) void k_store_lanes_wait(uint8_t *dst, uint64_t *out, uint32_t span, uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const uint32_t l = threadIdx.x, piece = l % 32;
    const u32x4 v = {l * 0x01010101u, blockIdx.x, 0xC3C3C3C3u, ~l};
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * 64ull * span;
        for (uint32_t it = 0; it < span / 512; ++it) {
            for (int i = 0; i < 32; ++i) st_sc1(base + (uint64_t)(2 * i + l / 32) * span + it * 512 + piece * 16, v);
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
        }
    }
    stamp(out, t0);
}

// one granule per workgroup with part of the fill's work in front of the
// stores: `work` Xoshiro steps (VALU) and/or (load != 0) the lane's four 16-B
// pieces of a 4 KiB block read from L2 first, as the fill reads its base block
__global__ __launch_bounds__(64) void k_store_granule_work(uint8_t *dst, uint64_t *out, const u32x4 *blk, uint32_t work,
                                                           uint32_t load) {
    const uint64_t t0 = wall_clock64();
    u32x4 v = {threadIdx.x * 0x01010101u, blockIdx.x, 0x96969696u, ~threadIdx.x};
    uint64_t s0 = threadIdx.x + 1, s1 = blockIdx.x * 77 + 3, s2 = 0x9E3779B97F4A7C15ull, s3 = 12345;
    for (uint32_t i = 0; i < work; ++i) {
        const uint64_t t = s1 << 17;
        s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45);
    }
    v.x ^= (uint32_t)(s0 + s3);
    u32x4 b[4] = {v, v, v, v};
    if (load)
        for (int i = 0; i < 4; ++i) b[i] = blk[threadIdx.x + 64 * i] ^ v;
    const uint64_t g = blockIdx.x;
    for (int i = 0; i < 4; ++i) st_sc1(dst + g * 4096 + threadIdx.x * 16 + 1024 * i, b[i]);
    stamp(out, t0);
}

// the lane pattern, each 32-store burst's data XOR-ed with the lane's 16 B of
// an L2-resident block read just before it (the burst waits for that read)
__global__ __launch_bounds__(64) void k_store_lanes_load(uint8_t *dst, uint64_t *out, const u32x4 *blk, uint32_t span,
                                                         uint32_t units) {
    const uint64_t t0 = wall_clock64();
    const uint32_t l = threadIdx.x, piece = l % 32;
    const u32x4 v = {l * 0x01010101u, blockIdx.x, 0xE1E1E1E1u, ~l};
    for (uint32_t u = 0; u < units; ++u) {
        uint8_t *base = dst + ((uint64_t)u * gridDim.x + blockIdx.x) * 64ull * span;
        for (uint32_t it = 0; it < span / 512; ++it) {
            const u32x4 b = blk[(l + it) & 255] ^ v;
            for (int i = 0; i < 32; ++i) st_sc1(base + (uint64_t)(2 * i + l / 32) * span + it * 512 + piece * 16, b);
        }
    }
    stamp(out, t0);
}

extern "C" {
int lab_store_lanes_load(void *dst, void *out, const void *blk, uint32_t grid, uint32_t span, uint32_t units,
                         uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_lanes_load, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out,
                       (const u32x4 *)blk, span, units);
    return (int)hipGetLastError();
}
int lab_store_granule_work(void *dst, void *out, const void *blk, uint32_t grid, uint32_t work, uint32_t load,
                           uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_granule_work, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst,
                       (uint64_t *)out, (const u32x4 *)blk, work, load);
    return (int)hipGetLastError();
}
int lab_store_lanes_wait(void *dst, void *out, uint32_t grid, uint32_t span, uint32_t units, uint32_t n, uint32_t lds,
                         void *s) {
    if (n == 0)
        hipLaunchKernelGGL(k_store_lanes_wait<0>, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst,
                           (uint64_t *)out, span, units);
    else if (n == 16)
        hipLaunchKernelGGL(k_store_lanes_wait<16>, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst,
                           (uint64_t *)out, span, units);
    else
        hipLaunchKernelGGL(k_store_lanes_wait<32>, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst,
                           (uint64_t *)out, span, units);
    return (int)hipGetLastError();
}
int lab_store_granule(void *dst, void *out, uint32_t grid, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_granule, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out);
    return (int)hipGetLastError();
}
int lab_store_lanes_rnd(void *dst, void *out, uint32_t grid, uint32_t span, uint32_t units, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_lanes_rnd, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out,
                       span, units);
    return (int)hipGetLastError();
}
int lab_store_window(void *dst, void *out, uint32_t grid, uint64_t ngran, uint32_t nap, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_window, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out,
                       ngran, nap);
    return (int)hipGetLastError();
}
int lab_store_lanes_paced(void *dst, void *out, uint32_t grid, uint32_t span, uint32_t units, uint32_t nap,
                          uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_lanes_paced, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst,
                       (uint64_t *)out, span, units, nap);
    return (int)hipGetLastError();
}
int lab_store_xcd(void *dst, void *out, uint32_t grid, uint32_t units, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_xcd, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out, units);
    return (int)hipGetLastError();
}
int lab_valu(void *out, void *sink, uint32_t grid, uint32_t iters, void *s) {
    hipLaunchKernelGGL(k_valu, dim3(grid), dim3(64), 0, (hipStream_t)s, (uint64_t *)out, (uint64_t *)sink, iters);
    return (int)hipGetLastError();
}
int lab_store_seq(void *dst, void *out, uint32_t grid, uint64_t bpw, uint32_t units, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_seq, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out, bpw,
                       units);
    return (int)hipGetLastError();
}
int lab_store_lanes(void *dst, void *out, uint32_t grid, uint32_t span, uint32_t units, uint32_t lds, void *s) {
    hipLaunchKernelGGL(k_store_lanes, dim3(grid), dim3(64), lds, (hipStream_t)s, (uint8_t *)dst, (uint64_t *)out,
                       span, units);
    return (int)hipGetLastError();
}
}
