// reg_fill_lab.hip — diagnostic kernels (tools/reg_fill_lab.py; not product
// code): how much of config 2's power and time goes to the fill's on-chip
// data movement (the base block read from L2 and the LDS image) rather than
// to the HBM stores.  All kernels store the 4 KiB base block (random bytes,
// so the HBM data toggles like the fill's) into every 4 KiB granule of dst:
//   k_store_l2   one 64-thread workgroup per granule, each lane loads its four
//                16-B base pieces from L2 and stores them (no LDS)
//   k_store_lds  the same through an LDS image and a barrier (the fill's
//                shape without the PRNG chain and the window patches)
//   k_store_reg  a persistent grid: each lane loads its pieces once and stores
//                them into granules b, b + R, b + 2R, ... (R = grid size, a
//                multiple of 8, so a workgroup on XCD b mod 8 keeps to the
//                granules = b (mod 8), as the fill); `spin` s_sleep units
//                between granules pace it
// Stores are global_store_dwordx4 ... sc1, as the fill's.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1(uint8_t *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}

__global__ __launch_bounds__(64) void k_store_l2(uint8_t *dst, const u32x4 *base, uint64_t nblk) {
    const uint64_t g = blockIdx.x;
    if (g >= nblk) return;
    const uint32_t t = threadIdx.x;
    u32x4 B[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) B[k] = base[t + 64 * k];
    uint8_t *p = dst + g * 4096 + t * 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) st_sc1(p + 1024 * k, B[k]);
}

__global__ __launch_bounds__(64) void k_store_lds(uint8_t *dst, const u32x4 *base, uint64_t nblk) {
    __shared__ __attribute__((aligned(16))) uint8_t img[4096];
    const uint64_t g = blockIdx.x;
    if (g >= nblk) return;
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<u32x4 *>(img + 16 * (t + 64 * k)) = base[t + 64 * k];
    __syncthreads();
    uint8_t *p = dst + g * 4096 + t * 16;
#pragma unroll
    for (int k = 0; k < 4; ++k) st_sc1(p + 1024 * k, *reinterpret_cast<const u32x4 *>(img + 16 * (t + 64 * k)));
}

__global__ __launch_bounds__(64) void k_store_reg(uint8_t *dst, const u32x4 *base, uint64_t nblk, uint32_t spin) {
    const uint32_t t = threadIdx.x;
    u32x4 B[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) B[k] = base[t + 64 * k];
    const uint64_t R = gridDim.x;
    for (uint64_t g = blockIdx.x; g < nblk; g += R) {
        uint64_t off = g * 4096 + t * 16;
        asm volatile("" : "+v"(off));
        uint8_t *p = dst + off;
#pragma unroll
        for (int k = 0; k < 4; ++k) st_sc1(p + 1024 * k, B[k]);
        for (uint32_t s = 0; s < spin; ++s) __builtin_amdgcn_s_sleep(1);
    }
}

extern "C" {
int lab_store_l2(void *dst, const void *base, uint64_t nblk, uint32_t lds, void *stream) {
    hipLaunchKernelGGL(k_store_l2, dim3((uint32_t)nblk), dim3(64), lds, (hipStream_t)stream, (uint8_t *)dst,
                       (const u32x4 *)base, nblk);
    return (int)hipGetLastError();
}
int lab_store_lds(void *dst, const void *base, uint64_t nblk, uint32_t lds, void *stream) {
    hipLaunchKernelGGL(k_store_lds, dim3((uint32_t)nblk), dim3(64), lds, (hipStream_t)stream, (uint8_t *)dst,
                       (const u32x4 *)base, nblk);
    return (int)hipGetLastError();
}
int lab_store_reg(void *dst, const void *base, uint64_t nblk, uint32_t grid, uint32_t lds, uint32_t spin,
                  void *stream) {
    hipLaunchKernelGGL(k_store_reg, dim3(grid), dim3(64), lds, (hipStream_t)stream, (uint8_t *)dst,
                       (const u32x4 *)base, nblk, spin);
    return (int)hipGetLastError();
}
}
