// s3dg_crc.hip — CRC-32 (IEEE 802.3, reflected 0xEDB88320; crc32fast /
// zlib.crc32) of device buffers, for the NPZ builder
// (generate_npz_bytes_raw: crc32fast::hash over x.npy, src/data_formats/npz.rs:385-386)
// and the TFRecord / streaming-writer checksums (src/data_formats/tfrecord.rs:10-32,
// src/streaming_writer.rs:183-186).
//
// CRC is affine over GF(2), so pieces combine as in zlib's crc32_combine:
//   crc(A || B) = multmodp(x^(8|B|) mod P, crc(A)) ^ crc(B).
// Kernel: one wave per contiguous region (256 KiB by default), column-Horner
// (k_crc32_regions); the host folds the region CRCs (table-driven constant
// multiply) and hashes the sub-region tail itself.  Reads only: HBM-read bound.
#include "s3dg_internal.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace s3dg {
namespace {

constexpr uint32_t kPoly = 0xEDB88320u;

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

// Register-shift tables.  raw(M) is the CRC register after M from a zero
// register (linear in M); A^k is "advance k zero bytes" = multmodp(x^(8k), .).
//   Tbyte[k][x] = A^k(raw of the single byte x)     k = 0..15 (slicing-by-16)
//   Trow[b][x]  = A^1024(x << 8b)                     (multiply by x^(8*1024))
struct CrcTables {
    uint32_t tbyte[16][256];
    uint32_t trow[4][256];
};

__device__ __forceinline__ uint32_t mul_row(const uint32_t (*T)[256], uint32_t v) {
    return T[0][v & 0xFF] ^ T[1][(v >> 8) & 0xFF] ^ T[2][(v >> 16) & 0xFF] ^ T[3][v >> 24];
}

// One wave per region.  Segment s (s = 0..nseg-1) starts at src + s*seg_stride
// and holds seg_rows whole 1 KiB rows; region k of a segment covers rows
// [k*rows, min((k+1)*rows, seg_rows)).  Lane l owns bytes [16 l, 16 l + 16) of
// every row: each row is one coalesced 1 KiB load, and the lane keeps the
// Horner sum
//   S_l = A^1024 S_l ^ raw16(piece)
// so the region's raw CRC is XOR_l A^(16 (63 - l)) S_l.  Output: raw CRC per region.
struct CrcSegArgs {
    const uint8_t *src;
    uint64_t nreg;          // nseg * regs_per_seg
    uint64_t regs_per_seg;
    uint64_t seg_stride;    // bytes
    uint64_t seg_rows;      // whole 1 KiB rows per segment
    uint32_t rows;          // rows per region
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // gfx950 3-input LUT op: a ^ b ^ c
}

// 20 table words per row folded by a tree of 3-input XORs: 10 VALU ops
// instead of a serial chain of 19 two-input ones, and no long dependency
// chain behind the row-advance lookups (PMC: the kernel is issue-bound with
// no LDS bank conflicts, profiles/r02/diag/pmc_crc*).
__device__ __forceinline__ uint32_t horner_row(const uint32_t (*trow)[256], const uint32_t (*tbyte)[256],
                                               uint32_t S, const uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t t[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) t[q] = tbyte[15 - q][(w[q >> 2] >> (8 * (q & 3))) & 0xFF];
    const uint32_t a0 = xor3(t[0], t[1], t[2]), a1 = xor3(t[3], t[4], t[5]), a2 = xor3(t[6], t[7], t[8]);
    const uint32_t a3 = xor3(t[9], t[10], t[11]), a4 = xor3(t[12], t[13], t[14]);
    const uint32_t b0 = xor3(a0, a1, a2), b1 = xor3(a3, a4, t[15]);
    const uint32_t r0 = trow[0][S & 0xFF], r1 = trow[1][(S >> 8) & 0xFF], r2 = trow[2][(S >> 16) & 0xFF],
                   r3 = trow[3][S >> 24];
    return xor3(b0, b1, r0) ^ xor3(r1, r2, r3);
}

__global__ __launch_bounds__(256) void k_crc32_regions(CrcSegArgs a, const CrcTables *tabs,
                                                       const uint32_t *lane_shift, uint32_t *out) {
    __shared__ CrcTables T;
    const uint32_t t = threadIdx.x, lane = t & 63;
    {
        const uint32_t *g = reinterpret_cast<const uint32_t *>(tabs);
        uint32_t *d = reinterpret_cast<uint32_t *>(&T);
        for (uint32_t k = t; k < sizeof(CrcTables) / 4; k += 256) d[k] = g[k];
    }
    __syncthreads();
    const uint32_t (*trow)[256] = T.trow;
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (t >> 6);
    if (r >= a.nreg) return;
    const uint64_t seg = r / a.regs_per_seg, k = r - seg * a.regs_per_seg;
    const uint64_t row0 = k * a.rows;
    const uint32_t nrows = (uint32_t)((a.seg_rows - row0) < a.rows ? (a.seg_rows - row0) : a.rows);
    const uint4 *p = reinterpret_cast<const uint4 *>(a.src + seg * a.seg_stride + row0 * 1024) + lane;
    uint32_t S = 0, row = 0;
    // Software pipelined over two register buffers: while rows r..r+3 (A) are
    // hashed, rows r+4..r+7 (B) are in flight, then the other way round, so a
    // wave keeps 8 KiB outstanding and every row waits only for its own load.
    // The last loads of the loop are clamped to valid rows and not used.
    // sched_barrier keeps the compiler from sinking the loads into the hash.
    auto load4 = [&](uint4 (&v)[4], uint32_t r0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = r0 + q < nrows ? r0 + q : nrows - 1;
            v[q] = p[r * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    uint4 A[4], B[4];
    if (nrows >= 4) load4(A, 0);
    for (; row + 8 <= nrows; row += 8) {
        load4(B, row + 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) S = horner_row(trow, T.tbyte, S, A[q]);
        __builtin_amdgcn_sched_barrier(0);
        load4(A, row + 8);
#pragma unroll
        for (int q = 0; q < 4; ++q) S = horner_row(trow, T.tbyte, S, B[q]);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (row + 4 <= nrows) {
#pragma unroll
        for (int q = 0; q < 4; ++q) S = horner_row(trow, T.tbyte, S, A[q]);
        row += 4;
    }
    for (; row < nrows; ++row) S = horner_row(trow, T.tbyte, S, p[row * 64]);
    S = multmodp(lane_shift[lane], S);              // A^(16 (63 - lane))
#pragma unroll
    for (int q = 32; q >= 1; q >>= 1) S ^= __shfl_xor(S, q);
    if (lane == 0) out[r] = S;
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
CrcTables dev_tables_host;
uint32_t lane_shift_host[64];

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
    // raw CRC of one byte x is crc_tables[0][x]; A^k of it by k zero-byte steps
    for (uint32_t x = 0; x < 256; ++x) {
        uint32_t c = crc_tables[0][x];
        for (int k = 0; k < 16; ++k) {
            dev_tables_host.tbyte[k][x] = c;
            c = (c >> 8) ^ crc_tables[0][c & 0xFF];
        }
    }
    const uint32_t x1k = x8n(1024);
    for (int b = 0; b < 4; ++b)
        for (uint32_t x = 0; x < 256; ++x) dev_tables_host.trow[b][x] = multmodp(x1k, x << (8 * b));
    for (int l = 0; l < 64; ++l) lane_shift_host[l] = x8n(16ull * (63 - l));
    tables_ready = true;
}

}  // namespace

uint32_t crc32_host_update(uint32_t crc, const uint8_t *p, uint64_t n) {
    {
        static std::mutex m;
        std::lock_guard<std::mutex> g(m);
        init_tables();
    }
    uint32_t c = ~crc;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {                      // slicing-by-8 (little-endian host)
        uint32_t a, b;
        memcpy(&a, p + i, 4);
        memcpy(&b, p + i + 4, 4);
        a ^= c;
        c = crc_tables[7][a & 0xFF] ^ crc_tables[6][(a >> 8) & 0xFF] ^ crc_tables[5][(a >> 16) & 0xFF] ^
            crc_tables[4][a >> 24] ^ crc_tables[3][b & 0xFF] ^ crc_tables[2][(b >> 8) & 0xFF] ^
            crc_tables[1][(b >> 16) & 0xFF] ^ crc_tables[0][b >> 24];
    }
    for (; i < n; ++i) c = (c >> 8) ^ crc_tables[0][(c ^ p[i]) & 0xFF];
    return ~c;
}

uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return multmodp(x8n(len2), crc1) ^ crc2;
}

hipError_t crc_tables_device(void **tab_cache) {
    static std::mutex init_mu;
    {
        std::lock_guard<std::mutex> g(init_mu);
        init_tables();
    }
    if (*tab_cache) return hipSuccess;
    hipError_t e;
    if ((e = hipMalloc(tab_cache, sizeof(CrcTables) + 64 * 4)) != hipSuccess) return e;
    if ((e = hipMemcpy(*tab_cache, &dev_tables_host, sizeof(CrcTables), hipMemcpyHostToDevice)) != hipSuccess)
        return e;
    return hipMemcpy((uint8_t *)*tab_cache + sizeof(CrcTables), lane_shift_host, 64 * 4,
                     hipMemcpyHostToDevice);
}

CrcSegPlan crc_seg_plan(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride) {
    CrcSegPlan P{};
    P.nseg = nseg;
    P.seg_len = seg_len;
    P.seg_stride = seg_stride;
    P.seg_rows = seg_len / 1024;
    uint32_t rows = 256;                                   // 256 KiB per wave region
    while (nseg * ((P.seg_rows + rows - 1) / rows) > (1ull << 24)) rows *= 2;
    P.rows = rows;
    P.regs_per_seg = (P.seg_rows + rows - 1) / rows;
    P.nreg = nseg * P.regs_per_seg;
    return P;
}

hipError_t crc_seg_launch(const CrcSegPlan &P, const uint8_t *dev, void *tab_dev, uint32_t *out_dev,
                          hipStream_t s) {
    if (P.nreg == 0) return hipSuccess;
    CrcSegArgs a{dev, P.nreg, P.regs_per_seg, P.seg_stride, P.seg_rows, P.rows};
    const uint64_t wgs = (P.nreg + 3) / 4;
    (void)hipGetLastError();
    hipLaunchKernelGGL(k_crc32_regions, dim3((uint32_t)wgs), dim3(256), 0, s, a, (const CrcTables *)tab_dev,
                       (const uint32_t *)((uint8_t *)tab_dev + sizeof(CrcTables)), out_dev);
    return hipGetLastError();
}

// Fold region raw CRCs into per-segment CRC-32s.  tails[s] points at the
// segment's bytes past its whole rows (< 1 KiB, host memory), or is null when
// seg_len is a multiple of 1 KiB.
void crc_seg_fold(const CrcSegPlan &P, const uint32_t *regions, const uint8_t *const *tails,
                  uint32_t *crcs) {
    {
        static std::mutex m;
        std::lock_guard<std::mutex> g(m);
        init_tables();
    }
    const uint64_t region = (uint64_t)P.rows * 1024;
    const uint64_t last_rows = P.seg_rows - (P.regs_per_seg ? (P.regs_per_seg - 1) * P.rows : 0);
    uint32_t Tr[4][256];
    if (P.regs_per_seg > 1) {
        const uint32_t xr = x8n(region);
        for (int b = 0; b < 4; ++b)
            for (uint32_t x = 0; x < 256; ++x) Tr[b][x] = multmodp(xr, x << (8 * b));
    }
    const uint32_t x_last = x8n(last_rows * 1024);
    const uint64_t head = P.seg_rows * 1024, tail = P.seg_len - head;
    const uint32_t init = P.seg_rows ? multmodp(x8n(head), 0xFFFFFFFFu) : 0;
    for (uint64_t sg = 0; sg < P.nseg; ++sg) {
        uint32_t crc = 0;
        if (P.seg_rows) {
            const uint32_t *h = regions + sg * P.regs_per_seg;
            uint32_t raw = 0;
            for (uint64_t k = 0; k + 1 < P.regs_per_seg; ++k)
                raw = (Tr[0][raw & 0xFF] ^ Tr[1][(raw >> 8) & 0xFF] ^ Tr[2][(raw >> 16) & 0xFF] ^
                       Tr[3][raw >> 24]) ^ h[k];
            raw = multmodp(x_last, raw) ^ h[P.regs_per_seg - 1];
            crc = ~(init ^ raw);                          // std(M) = ~(A^n(~0) ^ raw(M))
        }
        if (tail) {
            const uint32_t ct = crc32_host_update(0, tails[sg], tail);
            crc = P.seg_rows ? crc32_combine(crc, ct, tail) : ct;
        }
        crcs[sg] = crc;
    }
}

// CRC-32 of dev[0, len) (one segment): device regions + host fold + host tail.
hipError_t crc32_device(const uint8_t *dev, uint64_t len, hipStream_t s, uint32_t *out,
                        void **tab_cache, uint32_t **seg_cache, uint64_t *seg_cap) {
    hipError_t e;
    if ((e = crc_tables_device(tab_cache)) != hipSuccess) return e;
    const CrcSegPlan P = crc_seg_plan(1, len, len);
    if (P.nreg > *seg_cap) {
        if (*seg_cache) (void)hipFree(*seg_cache);
        *seg_cache = nullptr;
        *seg_cap = 0;
        if ((e = hipMalloc(seg_cache, P.nreg * 4)) != hipSuccess) return e;
        *seg_cap = P.nreg;
    }
    if ((e = crc_seg_launch(P, dev, *tab_cache, *seg_cache, s)) != hipSuccess) return e;
    std::vector<uint32_t> h(P.nreg);
    if (P.nreg && (e = hipMemcpyAsync(h.data(), *seg_cache, P.nreg * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    const uint64_t head = P.seg_rows * 1024;
    std::vector<uint8_t> tb(len - head);
    if (!tb.empty() && (e = hipMemcpyAsync(tb.data(), dev + head, tb.size(), hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const uint8_t *tp = tb.data();
    crc_seg_fold(P, h.data(), &tp, out);
    return hipSuccess;
}

}  // namespace s3dg
