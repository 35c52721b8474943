// s3dg_crc.hip — CRC-32 (IEEE 802.3, reflected 0xEDB88320; crc32fast /
// zlib.crc32) of device buffers, for the NPZ builder
// (generate_npz_bytes_raw: crc32fast::hash over x.npy, src/data_formats/npz.rs:385-386)
// and the TFRecord / streaming-writer checksums (src/data_formats/tfrecord.rs:10-32,
// src/streaming_writer.rs:183-186).
//
// CRC is affine over GF(2), so pieces combine as in zlib's crc32_combine:
//   crc(A || B) = multmodp(x^(8|B|) mod P, crc(A)) ^ crc(B).
// Kernel: one 256-thread workgroup per segment of `seg_tiles` tiles of 16 KiB.
// Lane l of a tile hashes bytes [64 l, 64 l + 64) (slicing-by-8, tables in
// LDS), the 256 lane CRCs fold in a log-depth tree (shuffles within a wave,
// LDS across waves) with one constant x^(8 * 64 * 2^k) per level, and the
// workgroup folds its tiles in order.  The host folds the per-segment CRCs
// and hashes the sub-tile tail itself.  Reads only: HBM-read bound.
#include "s3dg_internal.h"

#include <cstring>
#include <vector>

namespace s3dg {
namespace {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kTile = 16384;       // bytes per tile = 256 lanes x 64 B

__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
    // a * b mod P in the reflected representation (x^0 = 0x80000000), as zlib
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

struct CrcConsts {
    uint32_t lvl[14];    // x^(8 * 64 * 2^k) mod P, k = 0..13 (64 B .. 512 KiB)
    uint32_t tile;       // x^(8 * 16384)
};

__global__ __launch_bounds__(256) void k_crc32_segments(const uint8_t *src, uint64_t ntiles,
                                                        uint32_t seg_tiles, const uint32_t *tables,
                                                        CrcConsts K, uint32_t *seg_crc) {
    __shared__ uint32_t T[8][256];
    __shared__ uint32_t wred[4];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (uint32_t k = t; k < 8 * 256; k += 256) (&T[0][0])[k] = tables[k];
    __syncthreads();
    const uint64_t tile0 = (uint64_t)blockIdx.x * seg_tiles;
    uint32_t acc = 0;           // CRC of the segment so far (crc of empty = 0)
    bool have = false;
    for (uint32_t q = 0; q < seg_tiles && tile0 + q < ntiles; ++q) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(src + (tile0 + q) * kTile + t * 64);
        uint32_t c = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < 16; k += 2) {            // slicing-by-8 over 64 bytes
            const uint32_t a = p[k] ^ c, b = p[k + 1];
            c = T[7][a & 0xFF] ^ T[6][(a >> 8) & 0xFF] ^ T[5][(a >> 16) & 0xFF] ^ T[4][a >> 24] ^
                T[3][b & 0xFF] ^ T[2][(b >> 8) & 0xFF] ^ T[1][(b >> 16) & 0xFF] ^ T[0][b >> 24];
        }
        c ^= 0xFFFFFFFFu;
        // fold lane pieces: level k merges pairs of 64*2^k-byte runs
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t right = __shfl_down(c, 1u << k);
            if ((lane & ((2u << k) - 1)) == 0) c = multmodp(K.lvl[k], c) ^ right;
        }
        if (lane == 0) wred[w] = c;                  // CRC of this wave's 4 KiB
        __syncthreads();
        if (t == 0) {
            uint32_t tc = wred[0];
            for (int k = 1; k < 4; ++k) tc = multmodp(K.lvl[6], tc) ^ wred[k];
            acc = have ? multmodp(K.tile, acc) ^ tc : tc;
            have = true;
        }
        __syncthreads();
    }
    if (t == 0) seg_crc[blockIdx.x] = acc;
}

// x^(8 n) mod P (zlib x2nmodp(n, 3)) on the host.
uint32_t x8n(uint64_t n) {
    uint32_t p = 1u << 31;           // x^0
    uint32_t sq = 1u << 30;          // x^1
    // square-and-multiply on the exponent 8n (as bits)
    uint64_t e = n * 8;              // n < 2^61
    while (e) {
        if (e & 1) p = multmodp(sq, p);
        sq = multmodp(sq, sq);
        e >>= 1;
    }
    return p;
}

uint32_t crc_tables[8][256];
bool tables_ready = false;

void init_tables() {
    if (tables_ready) return;
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        crc_tables[0][n] = c;
    }
    for (uint32_t n = 0; n < 256; ++n)
        for (int k = 1; k < 8; ++k)
            crc_tables[k][n] = (crc_tables[k - 1][n] >> 8) ^ crc_tables[0][crc_tables[k - 1][n] & 0xFF];
    tables_ready = true;
}

}  // namespace

uint32_t crc32_host_update(uint32_t crc, const uint8_t *p, uint64_t n) {
    init_tables();
    uint32_t c = ~crc;
    for (uint64_t i = 0; i < n; ++i) c = (c >> 8) ^ crc_tables[0][(c ^ p[i]) & 0xFF];
    return ~c;
}

uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return multmodp(x8n(len2), crc1) ^ crc2;
}

// CRC-32 of dev[0, len): device segments + host fold + host tail.
hipError_t crc32_device(const uint8_t *dev, uint64_t len, hipStream_t s, uint32_t *out,
                        void **tab_cache, uint32_t **seg_cache, uint64_t *seg_cap) {
    init_tables();
    const uint64_t ntiles = len / kTile;
    uint32_t crc = 0;
    hipError_t e = hipSuccess;
    if (ntiles) {
        if (!*tab_cache) {
            if ((e = hipMalloc(tab_cache, sizeof(crc_tables))) != hipSuccess) return e;
            if ((e = hipMemcpy(*tab_cache, crc_tables, sizeof(crc_tables), hipMemcpyHostToDevice)) != hipSuccess)
                return e;
        }
        // ~8 tiles (128 KiB) per workgroup, at most 2^20 segments
        uint32_t seg_tiles = 8;
        while ((ntiles + seg_tiles - 1) / seg_tiles > (1u << 20)) seg_tiles *= 2;
        const uint64_t nseg = (ntiles + seg_tiles - 1) / seg_tiles;
        if (nseg > *seg_cap) {
            if (*seg_cache) (void)hipFree(*seg_cache);
            *seg_cache = nullptr;
            *seg_cap = 0;
            if ((e = hipMalloc(seg_cache, nseg * 4)) != hipSuccess) return e;
            *seg_cap = nseg;
        }
        CrcConsts K;
        for (int k = 0; k < 14; ++k) K.lvl[k] = x8n(64ull << k);
        K.tile = x8n(kTile);
        hipLaunchKernelGGL(k_crc32_segments, dim3((uint32_t)nseg), dim3(256), 0, s, dev, ntiles,
                           seg_tiles, (const uint32_t *)*tab_cache, K, *seg_cache);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        std::vector<uint32_t> h(nseg);
        if ((e = hipMemcpyAsync(h.data(), *seg_cache, nseg * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        const uint64_t seg_bytes = (uint64_t)seg_tiles * kTile;
        const uint32_t xseg = x8n(seg_bytes);
        crc = h[0];
        for (uint64_t k = 1; k < nseg; ++k) {
            const uint64_t blen = (k + 1 < nseg) ? seg_bytes : (ntiles - k * seg_tiles) * kTile;
            crc = multmodp(blen == seg_bytes ? xseg : x8n(blen), crc) ^ h[k];
        }
    }
    const uint64_t tail = len - ntiles * kTile;
    if (tail) {
        std::vector<uint8_t> tb(tail);
        if ((e = hipMemcpyAsync(tb.data(), dev + ntiles * kTile, tail, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        crc = ntiles ? crc32_combine(crc, crc32_host_update(0, tb.data(), tail), tail)
                     : crc32_host_update(0, tb.data(), tail);
    }
    *out = crc;
    return hipSuccess;
}

}  // namespace s3dg
