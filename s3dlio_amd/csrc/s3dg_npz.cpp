// s3dg_npz.cpp — generate_npz_bytes_raw (src/data_formats/npz.rs:322-434) on
// the GPU: the x-array payload is the K2 keystream (npz.rs:376-383: 2 MiB
// chunks, chunk k seeded seed_from_u64(k)), its CRC-32 comes from the device
// CRC kernel (npz.rs:385-386); the NPY/ZIP framing is assembled on the host
// with the same byte layout (npz.rs:216-309, 331-431).
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace s3dg {
uint32_t crc32_host_update(uint32_t crc, const uint8_t *p, uint64_t n);
uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
hipError_t crc32_device(const uint8_t *dev, uint64_t len, hipStream_t s, uint32_t *out,
                        void **tab_cache, uint32_t **seg_cache, uint64_t *seg_cap);
}  // namespace s3dg

extern "C" int s3dg_internal_fail(int code, const char *msg);
struct s3dg_ctx;
extern "C" int s3dg_internal_ctx_device(s3dg_ctx *c, int *dev);

namespace {

using namespace s3dg;

// build_npy_header_typed (npz.rs:216-241): NPY 1.0, padded to 64 bytes.
std::vector<uint8_t> npy_header(const uint64_t *shape, int ndim, const std::string &dtype) {
    std::string dims;
    for (int i = 0; i < ndim; ++i) {
        if (i) dims += ", ";
        dims += std::to_string(shape[i]);
    }
    const std::string tuple = ndim == 1 ? "(" + dims + ",)" : "(" + dims + ")";
    const std::string dict = "{'descr': '" + dtype + "', 'fortran_order': False, 'shape': " + tuple + ", }";
    const size_t header_len = dict.size() + 1;
    const size_t padding = (64 - ((6 + 2 + 2 + header_len) % 64)) % 64;
    const uint16_t hdl = (uint16_t)(header_len + padding);
    std::vector<uint8_t> r = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0, (uint8_t)(hdl & 0xFF), (uint8_t)(hdl >> 8)};
    r.insert(r.end(), dict.begin(), dict.end());
    r.insert(r.end(), padding, ' ');
    r.push_back('\n');
    return r;
}

// dtype_element_size (npz.rs:244-252): last ASCII digit of the dtype, else 4.
uint64_t elem_size(const std::string &dtype) {
    for (auto it = dtype.rbegin(); it != dtype.rend(); ++it)
        if (*it >= '0' && *it <= '9') return (uint64_t)(*it - '0');
    return 4;
}

void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
void put32(uint8_t *p, uint32_t v) { for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (8 * k)); }

// write_local_file_header (npz.rs:256-270)
void local_header(uint8_t *d, const char *name, uint32_t crc, uint32_t size) {
    const uint16_t n = (uint16_t)strlen(name);
    memcpy(d, "PK\x03\x04", 4);
    put16(d + 4, 20); put16(d + 6, 0); put16(d + 8, 0); put16(d + 10, 0); put16(d + 12, 0);
    put32(d + 14, crc); put32(d + 18, size); put32(d + 22, size);
    put16(d + 26, n); put16(d + 28, 0);
    memcpy(d + 30, name, n);
}

// write_central_dir_entry (npz.rs:273-297)
void central_entry(uint8_t *d, const char *name, uint32_t size, uint32_t crc, uint32_t off) {
    const uint16_t n = (uint16_t)strlen(name);
    memcpy(d, "PK\x01\x02", 4);
    put16(d + 4, 20); put16(d + 6, 20); put16(d + 8, 0); put16(d + 10, 0); put16(d + 12, 0);
    put16(d + 14, 0); put32(d + 16, crc); put32(d + 20, size); put32(d + 24, size);
    put16(d + 28, n); put16(d + 30, 0); put16(d + 32, 0); put16(d + 34, 0); put16(d + 36, 0);
    put32(d + 38, 0); put32(d + 42, off);
    memcpy(d + 46, name, n);
}

// write_eocd (npz.rs:300-309)
void eocd(uint8_t *d, uint16_t entries, uint32_t cd_size, uint32_t cd_off) {
    memcpy(d, "PK\x05\x06", 4);
    put16(d + 4, 0); put16(d + 6, 0); put16(d + 8, entries); put16(d + 10, entries);
    put32(d + 12, cd_size); put32(d + 16, cd_off); put16(d + 20, 0);
}

struct Layout {
    std::vector<uint8_t> hx, hy;
    uint64_t x_data, y_data, x_npy, y_npy;
    uint64_t off_x_npy, off_x_data, off_y_local, off_y_npy, off_y_data, off_cd, off_cd_y, off_eocd, total;
};

// exact offsets of npz.rs:331-363
Layout layout(const uint64_t *shape, int ndim, const std::string &dtype, uint64_t num_samples) {
    Layout L;
    L.hx = npy_header(shape, ndim, dtype);
    const uint64_t ys[1] = {num_samples};
    L.hy = npy_header(ys, 1, "<i8");
    uint64_t prod = 1;
    for (int i = 0; i < ndim; ++i) prod *= shape[i];
    L.x_data = prod * elem_size(dtype);
    L.y_data = num_samples * 8;
    L.x_npy = L.hx.size() + L.x_data;
    L.y_npy = L.hy.size() + L.y_data;
    L.off_x_npy = 30 + 5;
    L.off_x_data = L.off_x_npy + L.hx.size();
    L.off_y_local = L.off_x_data + L.x_data;
    L.off_y_npy = L.off_y_local + 30 + 5;
    L.off_y_data = L.off_y_npy + L.hy.size();
    L.off_cd = L.off_y_data + L.y_data;
    L.off_cd_y = L.off_cd + 46 + 5;
    L.off_eocd = L.off_cd_y + 46 + 5;
    L.total = L.off_eocd + 22;
    return L;
}

}  // namespace

struct s3dg_ctx;
extern "C" {
int s3dg_xoshiro_fill(s3dg_ctx *ctx, void *dst, uint64_t len, uint64_t chunk_bytes, uint64_t seed_base,
                      void *stream);
int s3dg_internal_crc_device(s3dg_ctx *ctx, const void *dev, uint64_t len, void *stream, uint32_t *out);

int s3dg_npz_size(const uint64_t *shape, int ndim, const char *dtype, uint64_t num_samples,
                  uint64_t *total) {
    if (!total || ndim < 0 || (ndim > 0 && !shape) || !dtype)
        return s3dg_internal_fail(S3DG_EINVAL, "bad npz arguments");
    *total = layout(shape, ndim, dtype, num_samples).total;
    return S3DG_OK;
}

int s3dg_npz_build(s3dg_ctx *ctx, const uint64_t *shape, int ndim, const char *dtype,
                   uint64_t num_samples, uint8_t *out, uint64_t out_len) {
    if (!ctx || !out || ndim < 0 || (ndim > 0 && !shape) || !dtype)
        return s3dg_internal_fail(S3DG_EINVAL, "bad npz arguments");
    const Layout L = layout(shape, ndim, dtype, num_samples);
    if (out_len < L.total) return s3dg_internal_fail(S3DG_EINVAL, "output buffer too small");
    uint32_t crc_x = crc32_host_update(0, L.hx.data(), L.hx.size());
    if (L.x_data) {
        // cached grow-only device buffer + stream per device (one build at a
        // time per device)
        struct Cache {
            std::mutex mu;
            void *dev = nullptr;
            uint64_t cap = 0;
            hipStream_t s = nullptr, s_crc = nullptr;   // D2H stream, CRC stream
            hipEvent_t filled = nullptr;
            void *crc_tab = nullptr;                     // CRC tables (device)
            uint32_t *reg = nullptr;                     // region CRCs (device)
            uint64_t reg_cap = 0;
        };
        static std::mutex map_mu;
        static std::map<int, Cache *> *caches = new std::map<int, Cache *>();   // never freed: outlives HIP
        int device = 0;
        if (int r = s3dg_internal_ctx_device(ctx, &device)) return r;
        DeviceScope ds(device);
        if (!ds.ok()) return s3dg_internal_fail(S3DG_EHIP, "hipSetDevice");
        Cache *C;
        {
            std::lock_guard<std::mutex> g(map_mu);
            Cache *&slot = (*caches)[device];
            if (!slot) slot = new Cache();
            C = slot;
        }
        std::lock_guard<std::mutex> lk(C->mu);
        void *&dev = C->dev;
        uint64_t &cap = C->cap;
        hipStream_t &s = C->s;
        if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
            return s3dg_internal_fail(S3DG_EHIP, "hipStreamCreate");
        if (!C->s_crc && hipStreamCreateWithFlags(&C->s_crc, hipStreamNonBlocking) != hipSuccess)
            return s3dg_internal_fail(S3DG_EHIP, "hipStreamCreate");
        if (!C->filled && hipEventCreateWithFlags(&C->filled, hipEventDisableTiming) != hipSuccess)
            return s3dg_internal_fail(S3DG_EHIP, "hipEventCreate");
        if (L.x_data > cap) {
            if (dev) (void)hipFree(dev);
            dev = nullptr;
            cap = 0;
            if (hipMalloc(&dev, L.x_data) != hipSuccess)
                return s3dg_internal_fail(S3DG_ENOMEM, "hipMalloc(npz x-data)");
            cap = L.x_data;
        }
        uint32_t cd = 0;
        // after a failure nothing may still read `dev` or write C->reg when the
        // next build reuses them: both streams are drained first
        auto bail = [&](int code, const char *msg) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamSynchronize(C->s_crc);
            return s3dg_internal_fail(code, msg);
        };
        if (int r = s3dg_xoshiro_fill(ctx, dev, L.x_data, 2u << 20, 0, s)) {
            const std::string m = s3dg_last_error();
            return bail(r, m.c_str());
        }   // :376-383
        // The D2H (PCIe) and the CRC kernel (HBM reads) both only read the
        // keystream: the CRC runs on a second stream, hidden under the copy.
        if (hipEventRecord(C->filled, s) != hipSuccess || hipStreamWaitEvent(C->s_crc, C->filled, 0) != hipSuccess)
            return bail(S3DG_EHIP, "npz event");
        // The CRC kernel is enqueued first on its own stream, then the D2H
        // (which, into pageable memory, returns only when done): the two
        // overlap on the GPU.  The region CRCs are fetched after the D2H, and
        // the < 1 KiB tail is hashed from the host copy, so no two copies are
        // in flight from two host threads.
        if (crc_tables_device(&C->crc_tab) != hipSuccess) return bail(S3DG_EHIP, "crc tables");
        const CrcSegPlan P = crc_seg_plan(1, L.x_data, L.x_data);
        if (P.nreg > C->reg_cap) {
            (void)hipStreamSynchronize(C->s_crc);   // the previous build's CRC may still write it
            if (C->reg) (void)hipFree(C->reg);
            C->reg = nullptr;
            C->reg_cap = 0;
            if (hipMalloc(&C->reg, P.nreg * 4) != hipSuccess) return bail(S3DG_ENOMEM, "hipMalloc(crc)");
            C->reg_cap = P.nreg;
        }
        if (crc_seg_launch(P, (const uint8_t *)dev, C->crc_tab, C->reg, C->s_crc) != hipSuccess)
            return bail(S3DG_EHIP, "launch k_crc32_regions");
        if (hipMemcpyAsync(out + L.off_x_data, dev, L.x_data, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return bail(S3DG_EHIP, "npz x-data D2H");
        std::vector<uint32_t> regions(P.nreg);
        if (P.nreg && (hipMemcpyAsync(regions.data(), C->reg, P.nreg * 4, hipMemcpyDeviceToHost, C->s_crc) != hipSuccess ||
                       hipStreamSynchronize(C->s_crc) != hipSuccess))
            return bail(S3DG_EHIP, "npz crc regions");
        const uint8_t *tail = out + L.off_x_data + P.seg_rows * 1024;
        crc_seg_fold(P, regions.data(), &tail, &cd);
        crc_x = crc32_combine(crc_x, cd, L.x_data);                                    // :386
    }
    // x.npy: local header + NPY header (:368-372, patched :389-392)
    local_header(out, "x.npy", crc_x, (uint32_t)L.x_npy);
    memcpy(out + L.off_x_npy, L.hx.data(), L.hx.size());
    // y.npy: int64 zeros (:394-410)
    memcpy(out + L.off_y_npy, L.hy.data(), L.hy.size());
    memset(out + L.off_y_data, 0, L.y_data);
    const uint32_t crc_y = crc32_host_update(0, out + L.off_y_npy, L.y_npy);
    local_header(out + L.off_y_local, "y.npy", crc_y, (uint32_t)L.y_npy);
    // central directory + EOCD (:412-430)
    central_entry(out + L.off_cd, "x.npy", (uint32_t)L.x_npy, crc_x, 0);
    central_entry(out + L.off_cd_y, "y.npy", (uint32_t)L.y_npy, crc_y, (uint32_t)L.off_y_local);
    eocd(out + L.off_eocd, 2, (uint32_t)(46 + 5 + 46 + 5), (uint32_t)L.off_cd);
    return S3DG_OK;
}

}  // extern "C"
