// s3dg_object.cpp — object assembly (L4 of SURVEY.md §1): generate_object
// (src/data_gen.rs:29-94) = payload dispatch + format wrap, on top of the
// device generators.
//   payload:  !use_controlled -> generate_random_data (:66-69, :102-132; here the
//             seeded analogue k_fill_stream/random-data layout)
//             Streaming / SinglePass -> the dgen-contract generator (DG1, :40-64)
//   format:   RAW      build_raw        (src/data_formats/raw.rs:7-9)
//             TFRECORD build_tfrecord   (src/data_formats/tfrecord.rs:10-75), exact framing
//             NPZ      build_npz        (src/data_formats/npz.rs:92-132): "data.npy" in a
//                      stored ZIP; the zip crate's exact header fields are not
//                      reproducible here (parity unpinned), the archive is a valid
//                      ZIP that numpy.load reads
//             HDF5     error, as a build without the hdf5 feature (:75-87)
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <cstring>
#include <string>
#include <vector>


extern "C" int s3dg_internal_fail(int code, const char *msg);
extern "C" int s3dg_internal_random_host(uint8_t *buf, uint64_t len, uint64_t entropy,
                                         int use_process_base);

namespace {

using namespace s3dg;

inline uint32_t mask_crc(uint32_t crc) {          // tfrecord.rs:10-12
    return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}
inline void put32(uint8_t *p, uint32_t v) { for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (8 * k)); }
inline void put64(uint8_t *p, uint64_t v) { for (int k = 0; k < 8; ++k) p[k] = (uint8_t)(v >> (8 * k)); }
inline void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

// make_npy_header (npz.rs:92-109): '|u1', shape (n,), padded to 16 bytes.
std::vector<uint8_t> npy_header_u1(uint64_t n) {
    std::string dict = "{'descr': '|u1', 'fortran_order': False, 'shape': (" + std::to_string(n) + ",)}";
    const size_t with_nl = 10 + dict.size() + 1;
    dict.append((16 - (with_nl % 16)) % 16, ' ');
    dict.push_back('\n');
    std::vector<uint8_t> r = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0, 0, 0};
    put16(&r[8], (uint16_t)dict.size());
    r.insert(r.end(), dict.begin(), dict.end());
    return r;
}

constexpr const char *kNpyName = "data.npy";
constexpr uint64_t kNameLen = 8;

uint64_t npz_legacy_size(uint64_t elements, uint64_t data_len) {
    return 30 + kNameLen + npy_header_u1(elements).size() + data_len + 46 + kNameLen + 22;
}

}  // namespace

namespace s3dg {

// Framing around a payload of `len` bytes whose CRC-32 is `pcrc`:
//   TFRECORD (one record)  u64 len | masked_crc(len) || payload || masked_crc(payload)
//   NPZ (legacy)           local header | "data.npy" | NPY header || payload ||
//                          central directory | EOCD
//   RAW                    nothing
void object_frame(int type, uint64_t elements, uint64_t len, uint32_t pcrc, std::vector<uint8_t> &pre,
                  std::vector<uint8_t> &suf) {
    pre.clear();
    suf.clear();
    if (type == S3DG_OBJ_TFRECORD) {
        pre.resize(12);
        put64(pre.data(), len);
        put32(pre.data() + 8, mask_crc(crc32_host_update(0, pre.data(), 8)));   // tfrecord.rs:20-23
        suf.resize(4);
        put32(suf.data(), mask_crc(pcrc));                                      // :27-29
    } else if (type == S3DG_OBJ_NPZ) {
        const std::vector<uint8_t> h = npy_header_u1(elements);
        const uint64_t npy = h.size() + len;
        const uint32_t crc = crc32_combine(crc32_host_update(0, h.data(), h.size()), pcrc, len);
        pre.resize(30 + kNameLen);
        uint8_t *p = pre.data();                          // local file header
        memcpy(p, "PK\x03\x04", 4);
        put16(p + 4, 10); put16(p + 6, 0); put16(p + 8, 0); put16(p + 10, 0); put16(p + 12, 0x21);
        put32(p + 14, crc); put32(p + 18, (uint32_t)npy); put32(p + 22, (uint32_t)npy);
        put16(p + 26, kNameLen); put16(p + 28, 0);
        memcpy(p + 30, kNpyName, kNameLen);
        pre.insert(pre.end(), h.begin(), h.end());
        const uint64_t cd_off = pre.size() + len;
        suf.resize(46 + kNameLen + 22);
        p = suf.data();                                   // central directory
        memcpy(p, "PK\x01\x02", 4);
        put16(p + 4, 20); put16(p + 6, 10); put16(p + 8, 0); put16(p + 10, 0); put16(p + 12, 0);
        put16(p + 14, 0x21); put32(p + 16, crc); put32(p + 20, (uint32_t)npy); put32(p + 24, (uint32_t)npy);
        put16(p + 28, kNameLen); put16(p + 30, 0); put16(p + 32, 0); put16(p + 34, 0); put16(p + 36, 0);
        put32(p + 38, 0); put32(p + 42, 0);
        memcpy(p + 46, kNpyName, kNameLen);
        p += 46 + kNameLen;                               // end of central directory
        memcpy(p, "PK\x05\x06", 4);
        put16(p + 4, 0); put16(p + 6, 0); put16(p + 8, 1); put16(p + 10, 1);
        put32(p + 12, 46 + kNameLen); put32(p + 16, (uint32_t)cd_off); put16(p + 20, 0);
    }
}

}  // namespace s3dg

extern "C" {

int s3dg_build_tfrecord(uint64_t records, uint64_t record_size, const uint8_t *data, uint8_t *out,
                        uint8_t *index_out) {
    if (records && (!data || !out)) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    uint64_t off = 0;
    uint8_t lb[8];
    put64(lb, record_size);
    const uint32_t len_crc = mask_crc(crc32_host_update(0, lb, 8));   // tfrecord.rs:20-23
    for (uint64_t i = 0; i < records; ++i) {
        uint8_t *p = out + off;
        const uint8_t *d = data + i * record_size;
        memcpy(p, lb, 8);
        put32(p + 8, len_crc);
        if (p + 12 != d) memmove(p + 12, d, record_size);             // :26
        put32(p + 12 + record_size, mask_crc(crc32_host_update(0, p + 12, record_size)));   // :27-29
        if (index_out) {                                              // build_tfrecord_with_index :64-66
            put64(index_out + 16 * i, off);
            put64(index_out + 16 * i + 8, 16 + record_size);
        }
        off += 16 + record_size;
    }
    return S3DG_OK;
}

int s3dg_npz_legacy_size(uint64_t elements, uint64_t data_len, uint64_t *out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *out = npz_legacy_size(elements, data_len);
    return S3DG_OK;
}

int s3dg_build_npz(uint64_t elements, const uint8_t *data, uint64_t data_len, uint8_t *out,
                   uint64_t out_len) {
    const uint64_t total = npz_legacy_size(elements, data_len);
    if (!out || out_len < total || (data_len && !data)) return s3dg_internal_fail(S3DG_EINVAL, "bad buffer");
    std::vector<uint8_t> pre, suf;
    const uint64_t off_data = 30 + kNameLen + npy_header_u1(elements).size();
    if (out + off_data != data) memmove(out + off_data, data, data_len);
    s3dg::object_frame(S3DG_OBJ_NPZ, elements, data_len, crc32_host_update(0, out + off_data, data_len), pre, suf);
    memcpy(out, pre.data(), pre.size());
    memcpy(out + off_data + data_len, suf.data(), suf.size());
    return S3DG_OK;
}

int s3dg_object_size(int type, uint64_t elements, uint64_t element_size, uint64_t *out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    const uint64_t total = elements * element_size;       // :32
    switch (type) {
    case S3DG_OBJ_RAW: *out = total; return S3DG_OK;
    case S3DG_OBJ_TFRECORD: *out = elements * (16 + element_size); return S3DG_OK;
    case S3DG_OBJ_NPZ: *out = npz_legacy_size(elements, total); return S3DG_OK;
    case S3DG_OBJ_HDF5:
        return s3dg_internal_fail(S3DG_EINVAL, "HDF5 format is not available in this build");  // :75-87
    default: return s3dg_internal_fail(S3DG_EINVAL, "unknown object type");
    }
}

int s3dg_generate_object(int type, uint64_t elements, uint64_t element_size, int use_controlled,
                         uint64_t dedup, uint64_t compress, int mode, int has_seed, uint64_t seed,
                         uint8_t *out, uint64_t out_len, uint64_t *written) {
    uint64_t need = 0;
    if (int r = s3dg_object_size(type, elements, element_size, &need)) return r;
    if (!written) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    if (out_len < need || (need && !out)) return s3dg_internal_fail(S3DG_EINVAL, "output buffer too small");
    const uint64_t total = elements * element_size;
    // generate the payload in place where the format allows it, else in a scratch vector
    std::vector<uint8_t> tmp;
    uint8_t *payload = out;
    if (type == S3DG_OBJ_NPZ) payload = out + 30 + kNameLen + npy_header_u1(elements).size();
    else if (type == S3DG_OBJ_TFRECORD && elements != 1) { tmp.resize(total); payload = tmp.data(); }
    else if (type == S3DG_OBJ_TFRECORD) payload = out + 12;
    if (total) {
        int r;
        if (!use_controlled)                                               // :66-69
            r = s3dg_internal_random_host(payload, total, seed, has_seed ? 0 : 1);
        else {
            // Streaming (:40-51) and SinglePass (:52-64) produce the same
            // dgen-contract bytes here; `mode` only selects how the reference
            // staged them on the CPU.  dedup/compress 0 -> 1 (:108-109)
            (void)mode;
            r = s3dg_generate_data(payload, total, dedup, compress, has_seed, seed);
        }
        if (r) return r;
    }
    switch (type) {
    case S3DG_OBJ_RAW: break;                                              // build_raw
    case S3DG_OBJ_TFRECORD:
        if (int r = s3dg_build_tfrecord(elements, element_size, payload, out, nullptr)) return r;
        break;
    case S3DG_OBJ_NPZ:
        if (int r = s3dg_build_npz(elements, payload, total, out, out_len)) return r;
        break;
    }
    *written = need;
    return S3DG_OK;
}

}  // extern "C"
