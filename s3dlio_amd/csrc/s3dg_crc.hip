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

#include <cstdlib>
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

// ---- conflict-free form (k_crc32_regions_cf) ---------------------------------
// The 20 lookups per 16-B piece above are ds_read_b32 with data-dependent
// indices: 32 lanes of a half-wave pick random entries of the same 1 KiB
// table, i.e. random banks (bank = dword address mod 32), ~3-way conflicts on
// random data (profiles/r02/diag/crc: conflict cycles 2.04x the useful ones).
// Here every lane of a half-wave reads a different bank at every lookup:
//   * each table lives in ONE bank: entry i of single-bank table copy k is the
//     dword i * 32 + k (a 256-entry table = 256 rows of one bank);
//   * byte tables: 16 tables x 2 copies = 32 banks.  Lane l hashes its piece's
//     bytes in a lane-dependent order: its 4 words are rotated by
//     s = (l >> 2) & 3 (8 v_cndmask per row), and at step q it takes byte
//     ((q + l) & 3) of rotated word q >> 2, i.e. original byte
//     b = 4 ((q/4 + s) & 3) + ((q + l) & 3), looked up in table 15 - b, copy
//     (l >> 4) & 1.  Over lanes 0..15 (s, l & 3) takes all 16 values, so b does:
//     16 tables x 2 copies = 32 distinct banks per lookup;
//   * row-advance tables: 4 tables x 8 copies.  At step k lane l looks up byte
//     t = (k + l) & 3 of S in table t, copy (l >> 2) & 7: 32 distinct banks.
// XOR is order-free, so the sum is the same; the bytes match k_crc32_regions
// (and zlib) exactly.  64 KiB of LDS per workgroup: 8-wave workgroups, the
// grid sized to the chip, each wave looping over regions.
struct CrcTablesCF {
    uint32_t tb[256 * 32];   // byte tables: tb[i*32 + 2t + c] = tbyte[t][i]
    uint32_t tr[256 * 32];   // row tables:  tr[i*32 + 8t + c] = trow[t][i]
};

__global__ __launch_bounds__(512) void k_crc32_regions_cf(CrcSegArgs a, const CrcTablesCF *tabs,
                                                          const uint32_t *lane_shift, uint32_t *out) {
    __shared__ CrcTablesCF T;
    const uint32_t t = threadIdx.x, lane = t & 63;
    {
        const uint4 *g = reinterpret_cast<const uint4 *>(tabs);
        uint4 *d = reinterpret_cast<uint4 *>(&T);
        for (uint32_t k = t; k < sizeof(CrcTablesCF) / 16; k += 512) d[k] = g[k];
    }
    __syncthreads();
    // per-lane byte offsets (bytes) of the single-bank table copies, and the
    // in-word byte shifts of the rotated schedule
    const uint32_t s = (lane >> 2) & 3, cb = (lane >> 4) & 1, cr = (lane >> 2) & 7;
    uint32_t offb[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint32_t b = 4 * (((uint32_t)(q >> 2) + s) & 3) + (((uint32_t)q + lane) & 3);
        offb[q] = 4 * (2 * (15 - b) + cb);
    }
    uint32_t shb[4], offr[4], shr[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        shb[m] = 8 * (((uint32_t)m + lane) & 3);
        const uint32_t tt = ((uint32_t)m + lane) & 3;
        shr[m] = 8 * tt;
        offr[m] = 4 * (8 * tt + cr);
    }
    const bool rot2 = s & 2, rot1 = s & 1;
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(T.tb);
    const uint8_t *tr = reinterpret_cast<const uint8_t *>(T.tr);
    auto look = [&](const uint8_t *base, uint32_t byte, uint32_t off) -> uint32_t {
        return *reinterpret_cast<const uint32_t *>(base + (byte << 7) + off);
    };
    auto row = [&](uint32_t S, const uint4 v) -> uint32_t {
        // words rotated by s
        const uint32_t x0 = rot2 ? v.z : v.x, x1 = rot2 ? v.w : v.y, x2 = rot2 ? v.x : v.z, x3 = rot2 ? v.y : v.w;
        const uint32_t w[4] = {rot1 ? x1 : x0, rot1 ? x2 : x1, rot1 ? x3 : x2, rot1 ? x0 : x3};
        uint32_t u[20];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            u[q] = look(tb, __builtin_amdgcn_ubfe(w[q >> 2], shb[q & 3], 8), offb[q]);
#pragma unroll
        for (int m = 0; m < 4; ++m) u[16 + m] = look(tr, __builtin_amdgcn_ubfe(S, shr[m], 8), offr[m]);
        const uint32_t a0 = xor3(u[0], u[1], u[2]), a1 = xor3(u[3], u[4], u[5]), a2 = xor3(u[6], u[7], u[8]);
        const uint32_t a3 = xor3(u[9], u[10], u[11]), a4 = xor3(u[12], u[13], u[14]);
        const uint32_t a5 = xor3(u[15], u[16], u[17]), a6 = u[18] ^ u[19];
        return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6);
    };
    const uint64_t nwaves = (uint64_t)gridDim.x * 8;
    for (uint64_t r = (uint64_t)blockIdx.x * 8 + (t >> 6); r < a.nreg; r += nwaves) {
        const uint64_t seg = r / a.regs_per_seg, k = r - seg * a.regs_per_seg;
        const uint64_t row0 = k * a.rows;
        const uint32_t nrows = (uint32_t)((a.seg_rows - row0) < a.rows ? (a.seg_rows - row0) : a.rows);
        const uint4 *p = reinterpret_cast<const uint4 *>(a.src + seg * a.seg_stride + row0 * 1024) + lane;
        uint32_t S = 0, rw = 0;
        auto load4 = [&](uint4 (&v)[4], uint32_t r0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t rr = r0 + q < nrows ? r0 + q : nrows - 1;
                v[q] = p[rr * 64];
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        uint4 A[4], B[4];
        if (nrows >= 4) load4(A, 0);
        for (; rw + 8 <= nrows; rw += 8) {
            load4(B, rw + 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) S = row(S, A[q]);
            __builtin_amdgcn_sched_barrier(0);
            load4(A, rw + 8);
#pragma unroll
            for (int q = 0; q < 4; ++q) S = row(S, B[q]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (rw + 4 <= nrows) {
#pragma unroll
            for (int q = 0; q < 4; ++q) S = row(S, A[q]);
            rw += 4;
        }
        for (; rw < nrows; ++rw) S = row(S, p[rw * 64]);
        S = multmodp(lane_shift[lane], S);              // A^(16 (63 - lane))
#pragma unroll
        for (int q = 32; q >= 1; q >>= 1) S ^= __shfl_xor(S, q);
        if (lane == 0) out[r] = S;
    }
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
CrcTablesCF dev_tables_cf_host;
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
    for (uint32_t i = 0; i < 256; ++i) {
        for (int t = 0; t < 16; ++t)
            for (int c = 0; c < 2; ++c) dev_tables_cf_host.tb[i * 32 + 2 * t + c] = dev_tables_host.tbyte[t][i];
        for (int t = 0; t < 4; ++t)
            for (int c = 0; c < 8; ++c) dev_tables_cf_host.tr[i * 32 + 8 * t + c] = dev_tables_host.trow[t][i];
    }
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
    // [CrcTables][lane shifts, 256 B][CrcTablesCF]
    if ((e = hipMalloc(tab_cache, sizeof(CrcTables) + 64 * 4 + sizeof(CrcTablesCF))) != hipSuccess) return e;
    if ((e = hipMemcpy(*tab_cache, &dev_tables_host, sizeof(CrcTables), hipMemcpyHostToDevice)) != hipSuccess)
        return e;
    if ((e = hipMemcpy((uint8_t *)*tab_cache + sizeof(CrcTables), lane_shift_host, 64 * 4,
                       hipMemcpyHostToDevice)) != hipSuccess)
        return e;
    return hipMemcpy((uint8_t *)*tab_cache + sizeof(CrcTables) + 64 * 4, &dev_tables_cf_host, sizeof(CrcTablesCF),
                     hipMemcpyHostToDevice);
}

// 0: k_crc32_regions_cf (default), 1: k_crc32_regions (env S3DG_CRC_KERNEL=1; A/B only, same bytes)
int crc_kernel_choice() {
    static const int k = [] {
        const char *v = getenv("S3DG_CRC_KERNEL");
        return v && v[0] == '1' ? 1 : 0;
    }();
    return k;
}

CrcSegPlan crc_seg_plan(uint64_t nseg, uint64_t seg_len, uint64_t seg_stride) {
    CrcSegPlan P{};
    P.nseg = nseg;
    P.seg_len = seg_len;
    P.seg_stride = seg_stride;
    P.seg_rows = seg_len / 1024;
    uint32_t rows = 256;                                   // 256 KiB per wave region
    // smaller regions when 256 KiB ones would not give about one wave per
    // resident slot (4096): a 256 MiB PUT chunk or a 140 MiB NPZ archive
    // otherwise runs 1024 / 560 waves on 256 CUs (32 KiB minimum)
    const uint64_t total_rows = nseg * P.seg_rows;
    if (total_rows / rows < 4096) {
        const uint64_t r = total_rows / 4096;
        rows = (uint32_t)(r < 32 ? 32 : r);
    }
    while (nseg * ((P.seg_rows + rows - 1) / rows) > (1ull << 24)) rows *= 2;
    // one large segment: at most 4096 regions (about one per resident wave),
    // so the host folds a few thousand region CRCs, not one per 256 KiB
    // (16 GiB: 65 536 -> 4096)
    while (nseg == 1 && (P.seg_rows + rows - 1) / rows > 4096) rows *= 2;
    P.rows = rows;
    P.regs_per_seg = (P.seg_rows + rows - 1) / rows;
    P.nreg = nseg * P.regs_per_seg;
    return P;
}

hipError_t crc_seg_launch(const CrcSegPlan &P, const uint8_t *dev, void *tab_dev, uint32_t *out_dev,
                          hipStream_t s) {
    if (P.nreg == 0) return hipSuccess;
    CrcSegArgs a{dev, P.nreg, P.regs_per_seg, P.seg_stride, P.seg_rows, P.rows};
    const uint32_t *lsh = (const uint32_t *)((uint8_t *)tab_dev + sizeof(CrcTables));
    (void)hipGetLastError();
    if (crc_kernel_choice() == 0) {
        // conflict-free form: 8-wave workgroups, 2 per CU (64 KiB LDS each),
        // every wave looping over regions
        const uint64_t need = (P.nreg + 7) / 8;
        const uint32_t wgs = (uint32_t)(need < 512 ? need : 512);
        hipLaunchKernelGGL(k_crc32_regions_cf, dim3(wgs), dim3(512), 0, s, a,
                           (const CrcTablesCF *)((uint8_t *)tab_dev + sizeof(CrcTables) + 64 * 4), lsh, out_dev);
    } else {
        const uint64_t wgs = (P.nreg + 3) / 4;
        hipLaunchKernelGGL(k_crc32_regions, dim3((uint32_t)wgs), dim3(256), 0, s, a, (const CrcTables *)tab_dev, lsh,
                           out_dev);
    }
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
