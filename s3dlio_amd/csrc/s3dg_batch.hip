// s3dg_batch.hip — device side of the batch record layout:
// the exclusive scan that turns a sub-batch's descriptors into record offsets
// (hipCUB device scan over a transform of the 40-B descriptors).  Split from
// s3dg_kernels.hip so the library templates compile once.
#include <hipcub/hipcub.hpp>

#include "s3dg_internal.h"

namespace s3dg {
namespace {

// tile records of one object: its blocks behind `lead` dead slots (its 4 KiB
// granule mod 8, so every workgroup's slot = granule mod 8), rounded up to tiles
struct TileCount {
    uint64_t base;
    uint32_t tshift;
    __host__ __device__ uint64_t operator()(const s3dg_obj_desc &o) const {
        const uint64_t nb = (o.size + kBlk - 1) / kBlk;
        const uint64_t lead = ((base + o.dst_off) >> 12) & 7;
        return (nb + lead + (1ull << tshift) - 1) >> tshift;
    }
};

}  // namespace

hipError_t launch_batch_scan(const s3dg_obj_desc *d, uint64_t n, uint32_t tshift, uintptr_t base, uint64_t *rec_lo,
                             void *tmp, size_t *tmp_bytes, hipStream_t s) {
    hipcub::TransformInputIterator<uint64_t, TileCount, const s3dg_obj_desc *> it(d, TileCount{(uint64_t)base, tshift});
    if (n > 0x7FFFFFFFull) return hipErrorInvalidValue;
    return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, it, rec_lo, (int)n, s);
}

}  // namespace s3dg
