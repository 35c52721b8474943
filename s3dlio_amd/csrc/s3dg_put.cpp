// s3dg_put.cpp — the generator's consumer: per-object
// payloads generated on the GPU, checksummed on the GPU, copied into a pinned
// host ring and written to files by a pool of writer threads.
//
// Replaces, for file:// targets:
//   put_objects_with_random_data_and_type(_with_progress)  src/s3_utils.rs:1717-1750
//   put_objects_parallel_with_progress                      src/s3_utils.rs:1812-1868
//   FileSystemObjectStore::put (create parents, write)      src/file_store.rs:550-569
//   StreamingDataWriter checksum (crc32fast of the data)    src/streaming_writer.rs:95-96,183-186
// The reference generates ONE buffer and PUTs it to every URI (:1741); here
// object j gets its own payload, seeded object_entropy(seed_base, j).
//
// Pipeline (one call):
//   generator thread: chunk c -> device slot c&1 on stream c&1:
//       fill kernel(s) -> k_crc32_regions over the chunk's objects (region
//       CRCs written straight into pinned host slot c%kHostSlots); chunk
//       c+1's fill + CRC are enqueued on the other stream, then chunk c's
//       payload D2H into the host slot -> event; then it finishes chunk c-1
//     (event wait, CRC fold, framing) and queues its objects to the writers;
//     a host slot is reused only after every write from it has completed.
//   writer threads (max_in_flight): open/create, pwritev(prefix, payload,
//     suffix) straight from pinned memory, close.
// Objects larger than a slot are split into slot-sized pieces that share
// one open file; their CRCs are combined with crc32_combine.
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <array>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" int s3dg_internal_ctx_device(s3dg_ctx *c, int *dev);
extern "C" int s3dg_internal_dgen_chunk(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride,
                                        uint64_t n_objs, uint64_t blk_lo, uint64_t blk_hi, uint64_t dedup,
                                        uint32_t f_num, uint32_t f_den, uint64_t seed_base,
                                        uint64_t first_obj, void *stream);
extern "C" int s3dg_internal_fill_chunk(s3dg_ctx *c, void *dst, uint64_t obj_size, uint64_t stride,
                                        uint64_t n_objs, uint64_t blk_lo, uint64_t blk_hi,
                                        int random_layout, uint64_t dedup, uint32_t f_num,
                                        uint32_t f_den, uint64_t seed_base, uint64_t first_obj,
                                        void *stream);

namespace s3dg {
void object_frame(int type, uint64_t elements, uint64_t len, uint32_t pcrc, std::vector<uint8_t> &pre,
                  std::vector<uint8_t> &suf);
}  // namespace s3dg

namespace {

using namespace s3dg;

constexpr uint64_t kSlotBytes = 256ull << 20;   // device chunk / host slot (multiple of 1 MiB)
constexpr int kHostSlots = 4;
// one region per object plus at most 4096 more (crc_seg_plan sizes regions for ~4096)
constexpr uint64_t kMaxRegions = kSlotBytes / kBlk + 4096 + kSlotBytes / (256 * 1024) + 16;

// Process-wide buffers per (device, lane), created on first use and reused;
// a lane's pool is held (mutex) for the duration of a call.
struct PutPool {
    std::mutex mu;
    bool ready = false;
    int device = -1;
    void *dev[2] = {nullptr, nullptr};
    hipStream_t st[2] = {nullptr, nullptr};
    uint8_t *host[kHostSlots] = {};
    uint32_t *host_reg[kHostSlots] = {};
    hipEvent_t ev[kHostSlots] = {};
    void *crc_tab = nullptr;
};

PutPool &pool(int device, int lane) {
    // never destroyed: HIP may be torn down first at exit
    static std::mutex *mu = new std::mutex();
    static std::map<std::pair<int, int>, PutPool *> *pools = new std::map<std::pair<int, int>, PutPool *>();
    std::lock_guard<std::mutex> g(*mu);
    PutPool *&p = (*pools)[{device, lane}];
    if (!p) p = new PutPool();
    return *p;
}

#define PUT_HIP(expr, what)                                                                      \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return s3dg_internal_fail(S3DG_EHIP, (std::string(what) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

int pool_init(PutPool &P, int device) {
    if (P.ready && P.device == device) return S3DG_OK;
    if (P.ready) return s3dg_internal_fail(S3DG_EINVAL, "put pipeline already bound to another device");
    PUT_HIP(hipSetDevice(device), "hipSetDevice");
    for (int k = 0; k < 2; ++k) {
        PUT_HIP(hipMalloc(&P.dev[k], kSlotBytes), "hipMalloc(put chunk)");
        PUT_HIP(hipStreamCreateWithFlags(&P.st[k], hipStreamNonBlocking), "hipStreamCreate");
    }
    NumaScope numa(device);            // the pinned ring on the GPU's NUMA node
    for (int k = 0; k < kHostSlots; ++k) {
        PUT_HIP(hipHostMalloc((void **)&P.host[k], kSlotBytes, hipHostMallocDefault), "hipHostMalloc(put ring)");
        // written by the CRC kernel directly (pinned host memory is device-visible)
        PUT_HIP(hipHostMalloc((void **)&P.host_reg[k], kMaxRegions * 4, hipHostMallocDefault),
                "hipHostMalloc(put crc regions)");
        PUT_HIP(hipEventCreateWithFlags(&P.ev[k], hipEventDisableTiming), "hipEventCreate");
    }
    PUT_HIP(crc_tables_device(&P.crc_tab), "crc tables");
    P.device = device;
    P.ready = true;
    return S3DG_OK;
}

int mkdir_parents(const std::string &path) {
    for (size_t i = 1; i < path.size(); ++i) {
        if (path[i] != '/') continue;
        const std::string d = path.substr(0, i);
        if (mkdir(d.c_str(), 0755) != 0 && errno != EEXIST) return -1;
    }
    return 0;
}

int open_create(const char *path) {
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0 && errno == ENOENT) {                       // file_store.rs:562-564
        if (mkdir_parents(path) == 0) fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    }
    return fd;
}

bool write_all(int fd, struct iovec *iov, int n, uint64_t off) {
    while (n > 0) {
        const ssize_t w = pwritev(fd, iov, n, (off_t)off);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        off += (uint64_t)w;
        size_t left = (size_t)w;
        while (n > 0 && left >= iov->iov_len) {
            left -= iov->iov_len;
            ++iov;
            --n;
        }
        if (n > 0) {
            iov->iov_base = (uint8_t *)iov->iov_base + left;
            iov->iov_len -= left;
        }
    }
    return true;
}

struct OpenFile {                // shared by the pieces of one split object
    int fd = -1;
    ~OpenFile() {
        if (fd >= 0) close(fd);
    }
};

struct Job {
    const char *path = nullptr;
    std::shared_ptr<OpenFile> of;    // set for pieces of a split object
    std::vector<uint8_t> pre, suf;   // framing: pre at file offset 0, suf right after the data
    const uint8_t *data = nullptr;
    uint64_t len = 0, data_off = 0;  // payload bytes at file offset data_off
    int lane = 0, slot = -1;         // pinned ring slot of the payload (-1: none)
};

struct Writers {
    std::mutex mu;
    std::condition_variable cv_job, cv_slot;
    std::deque<Job> q;
    std::vector<std::array<int, kHostSlots>> outstanding;   // per lane, per ring slot
    bool closing = false;
    std::atomic<bool> failed{false};
    std::string err;
    std::atomic<uint64_t> bytes{0}, files{0};
    std::vector<std::thread> th;

    void fail(const std::string &m) {
        std::lock_guard<std::mutex> g(mu);
        if (!failed.exchange(true)) err = m;
    }

    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_job.wait(lk, [&] { return closing || !q.empty(); });
                if (q.empty()) return;
                j = std::move(q.front());
                q.pop_front();
            }
            if (!failed.load()) do_write(j);
            if (j.slot >= 0) {
                std::lock_guard<std::mutex> g(mu);
                if (--outstanding[j.lane][j.slot] == 0) cv_slot.notify_all();
            }
        }
    }

    void do_write(Job &j) {
        int fd = j.of ? j.of->fd : open_create(j.path);
        if (fd < 0) {
            fail(std::string("open ") + j.path + ": " + strerror(errno));
            return;
        }
        struct iovec iov[3];
        int n = 0;
        const bool pre_adjacent = !j.pre.empty() && j.data_off == j.pre.size();
        if (!j.pre.empty() && !pre_adjacent) {
            struct iovec p{j.pre.data(), j.pre.size()};
            if (!write_all(fd, &p, 1, 0)) {
                fail(std::string("write ") + j.path + ": " + strerror(errno));
                if (!j.of) close(fd);
                return;
            }
        }
        if (pre_adjacent) iov[n++] = {j.pre.data(), j.pre.size()};
        if (j.len) iov[n++] = {(void *)j.data, j.len};
        if (!j.suf.empty()) iov[n++] = {j.suf.data(), j.suf.size()};
        const uint64_t off = pre_adjacent ? 0 : j.data_off;
        uint64_t total = 0;
        for (int k = 0; k < n; ++k) total += iov[k].iov_len;
        if (n && !write_all(fd, iov, n, off)) fail(std::string("write ") + j.path + ": " + strerror(errno));
        if (!pre_adjacent) total += j.pre.size();
        bytes += total;
        if (!j.of) {
            if (close(fd) != 0) fail(std::string("close ") + j.path + ": " + strerror(errno));
            files += 1;
        }
    }

    void push(Job &&j) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (j.slot >= 0) ++outstanding[j.lane][j.slot];
            q.push_back(std::move(j));
        }
        cv_job.notify_one();
    }

    void wait_slot(int lane, int s) {
        std::unique_lock<std::mutex> lk(mu);
        cv_slot.wait(lk, [&] { return outstanding[lane][s] == 0; });
    }

    void finish() {
        {
            std::lock_guard<std::mutex> g(mu);
            closing = true;
        }
        cv_job.notify_all();
        for (auto &t : th) t.join();
        th.clear();
    }
};

// CPUs this process may use: the affinity mask, further limited by a cgroup v2
// CPU quota (cpu.max) when one is set.
uint32_t usable_cpus() {
    static const uint32_t n = [] {
        cpu_set_t set;
        uint32_t c = 0;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) c = (uint32_t)CPU_COUNT(&set);
        if (c == 0) c = std::thread::hardware_concurrency();
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            unsigned long long period = 0;
            if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
                const unsigned long long quota = strtoull(q, nullptr, 10);
                const uint32_t qc = (uint32_t)((quota + period - 1) / period);
                if (qc > 0 && qc < c) c = qc;
            }
            fclose(f);
        }
        return c ? c : 1u;
    }();
    return n;
}

struct ChunkDesc {
    uint64_t first_obj = 0, n_objs = 0;   // packed objects, or the object of a piece
    uint64_t off = 0, len = 0;            // piece byte range within the object (split objects)
    bool piece = false;
};

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct PutArgs {
    const char *const *paths;
    uint64_t n, size;
    int object_type, payload;
    uint64_t dedup;
    uint32_t f_num, f_den;
    uint64_t seed_base;
    uint32_t *crc_out;
    uint64_t pre_len;
};

void frame_job(const PutArgs &A, uint64_t j, uint32_t pcrc, Job &job) {
    object_frame(A.object_type, 1, A.size, pcrc, job.pre, job.suf);
    if (A.crc_out) {
        uint32_t c = crc32_host_update(0, job.pre.data(), job.pre.size());
        c = job.pre.empty() ? pcrc : crc32_combine(c, pcrc, A.size);
        if (!job.suf.empty()) c = crc32_combine(c, crc32_host_update(0, job.suf.data(), job.suf.size()), job.suf.size());
        A.crc_out[j] = c;
    }
}

// One lane: objects [j0, j1) on one device through its own pool: chunk c ->
// device slot c&1 / stream c&1 -> pinned host slot c % kHostSlots -> writers.
int run_lane(const PutArgs &A, s3dg_ctx *ctx, PutPool &P, int lane, uint64_t j0, uint64_t j1, Writers &W,
             double &gpu_wait) {
    const uint64_t size = A.size;
    const uint64_t stride = (size + kBlk - 1) / kBlk * kBlk;
    std::vector<ChunkDesc> chunks;
    if (stride <= kSlotBytes) {
        const uint64_t K = kSlotBytes / stride;
        for (uint64_t j = j0; j < j1; j += K) {
            ChunkDesc c;
            c.first_obj = j;
            c.n_objs = j1 - j < K ? j1 - j : K;
            c.len = size;
            chunks.push_back(c);
        }
    } else {
        for (uint64_t j = j0; j < j1; ++j)
            for (uint64_t off = 0; off < size; off += kSlotBytes) {
                ChunkDesc c;
                c.first_obj = j;
                c.n_objs = 1;
                c.off = off;
                c.len = size - off < kSlotBytes ? size - off : kSlotBytes;
                c.piece = true;
                chunks.push_back(c);
            }
    }
    const uint64_t nbD = (size + kDgenBlock - 1) / kDgenBlock;
    std::shared_ptr<OpenFile> cur_file;   // split object being written
    uint32_t cur_crc = 0;

    // Per chunk, in stream order on its device slot's stream: the fill, the
    // CRC kernel, the region CRCs to the host, then (enqueue_d2h) the payload
    // D2H and the completion event.  The next chunk's fill and CRC are
    // enqueued on the other stream BEFORE this chunk's payload D2H, so they
    // run under the copy even when the runtime returns from the D2H call only
    // once the copy is done (it does for blit copies; rocprof trace,
    // DESIGN.md §5.4).
    auto enqueue_gen = [&](uint64_t ci) -> int {
        const ChunkDesc &c = chunks[ci];
        const int ds = (int)(ci & 1), hs = (int)(ci % kHostSlots);
        hipStream_t s = P.st[ds];
        uint8_t *d = (uint8_t *)P.dev[ds];
        if (A.payload == S3DG_PAYLOAD_DGEN) {        // one launch for the whole chunk
            const uint64_t b0 = c.off / kDgenBlock, b1 = (c.off + c.len + kDgenBlock - 1) / kDgenBlock;
            if (int r = s3dg_internal_dgen_chunk(ctx, d, size, stride, c.n_objs, c.piece ? b0 : 0,
                                                 c.piece ? b1 : nbD, A.dedup, A.f_num, A.f_den, A.seed_base,
                                                 c.first_obj, s))
                return r;
        } else {
            const uint64_t b0 = c.off / kBlk, b1 = (c.off + c.len + kBlk - 1) / kBlk;
            if (int r = s3dg_internal_fill_chunk(ctx, d, size, stride, c.n_objs, b0, b1,
                                                 A.payload == S3DG_PAYLOAD_RANDOM, A.dedup, A.f_num, A.f_den,
                                                 A.seed_base, c.first_obj, s))
                return r;
        }
        const CrcSegPlan cp = crc_seg_plan(c.n_objs, c.len, stride);
        if (cp.nreg > kMaxRegions) return s3dg_internal_fail(S3DG_EINVAL, "crc region table overflow");
        // The kernel writes the region CRCs straight into the pinned host slot
        // (a few KiB over PCIe): no D2H call here, because the runtime returns
        // from a D2H call only when the copy is done (rocprof trace, DESIGN.md
        // §5.4), which would hold this thread until the fill and CRC finish.
        // host_reg[hs] was last read by complete(ci - kHostSlots), already done.
        PUT_HIP(crc_seg_launch(cp, d, P.crc_tab, P.host_reg[hs], s), "launch k_crc32_regions");
        return S3DG_OK;
    };
    auto enqueue_d2h = [&](uint64_t ci) -> int {
        const ChunkDesc &c = chunks[ci];
        const int ds = (int)(ci & 1), hs = (int)(ci % kHostSlots);
        hipStream_t s = P.st[ds];
        W.wait_slot(lane, hs);                             // writers done with chunk ci - kHostSlots
        const uint64_t bytes = (c.n_objs - 1) * stride + c.len;
        PUT_HIP(hipMemcpyAsync(P.host[hs], P.dev[ds], bytes, hipMemcpyDeviceToHost, s),
                "hipMemcpyAsync(D2H payload)");
        PUT_HIP(hipEventRecord(P.ev[hs], s), "hipEventRecord");
        return S3DG_OK;
    };

    auto complete = [&](uint64_t ci) -> int {
        const ChunkDesc &c = chunks[ci];
        const int hs = (int)(ci % kHostSlots);
        const double tw = now_s();
        PUT_HIP(hipEventSynchronize(P.ev[hs]), "hipEventSynchronize(put chunk)");
        gpu_wait += now_s() - tw;
        const CrcSegPlan cp = crc_seg_plan(c.n_objs, c.len, stride);
        std::vector<const uint8_t *> tails(c.n_objs);
        for (uint64_t k = 0; k < c.n_objs; ++k) tails[k] = P.host[hs] + k * stride + cp.seg_rows * 1024;
        std::vector<uint32_t> crcs(c.n_objs);
        crc_seg_fold(cp, P.host_reg[hs], tails.data(), crcs.data());
        if (!c.piece) {
            for (uint64_t k = 0; k < c.n_objs; ++k) {
                const uint64_t j = c.first_obj + k;
                Job job;
                job.path = A.paths[j];
                frame_job(A, j, crcs[k], job);
                job.data = P.host[hs] + k * stride;
                job.len = size;
                job.data_off = A.pre_len;
                job.lane = lane;
                job.slot = hs;
                W.push(std::move(job));
            }
            return S3DG_OK;
        }
        const uint64_t j = c.first_obj;
        if (c.off == 0) {
            cur_file = std::make_shared<OpenFile>();
            cur_file->fd = open_create(A.paths[j]);
            if (cur_file->fd < 0) {
                W.fail(std::string("open ") + A.paths[j] + ": " + strerror(errno));
                return S3DG_OK;
            }
            cur_crc = crcs[0];
        } else {
            cur_crc = crc32_combine(cur_crc, crcs[0], c.len);
        }
        Job job;
        job.path = A.paths[j];
        job.of = cur_file;
        job.data = P.host[hs];
        job.len = c.len;
        job.data_off = A.pre_len + c.off;
        job.lane = lane;
        job.slot = hs;
        if (c.off + c.len == size) {                       // last piece: framing with the full CRC
            frame_job(A, j, cur_crc, job);
            W.files += 1;                                  // closed when the last piece job drops it
            cur_file.reset();
        }
        W.push(std::move(job));
        return S3DG_OK;
    };

    int rc = S3DG_OK;
    if (!chunks.empty()) rc = enqueue_gen(0);
    for (uint64_t ci = 0; ci < chunks.size() && rc == S3DG_OK && !W.failed.load(); ++ci) {
        // chunk ci+1's fill + CRC (other stream) go in before chunk ci's payload
        // D2H; its device chunk was last copied out by chunk ci-1's D2H, earlier
        // on the same stream
        if (ci + 1 < chunks.size() && (rc = enqueue_gen(ci + 1)) != S3DG_OK) break;
        if ((rc = enqueue_d2h(ci)) != S3DG_OK) break;
        if (ci > 0) rc = complete(ci - 1);
    }
    if (rc == S3DG_OK && !W.failed.load() && !chunks.empty()) rc = complete(chunks.size() - 1);
    cur_file.reset();
    // drain the GPU before the pinned ring can be reused by the next call
    (void)hipStreamSynchronize(P.st[0]);
    (void)hipStreamSynchronize(P.st[1]);
    return rc;
}

}  // namespace

extern "C" int s3dg_put_objects_multi(s3dg_ctx *const *ctxs, uint32_t nctx, const char *const *paths,
                                      uint64_t n, uint64_t size, int object_type, int payload, uint64_t dedup,
                                      uint32_t f_num, uint32_t f_den, uint64_t seed_base,
                                      uint32_t max_in_flight, uint32_t *crc_out, s3dg_put_stats *stats) {
    const double t0 = now_s();
    if (!ctxs || nctx == 0) return s3dg_internal_fail(S3DG_EINVAL, "no context");
    if (nctx > 64) return s3dg_internal_fail(S3DG_EINVAL, "at most 64 contexts");
    for (uint32_t k = 0; k < nctx; ++k)
        if (!ctxs[k]) return s3dg_internal_fail(S3DG_EINVAL, "null context");
    if (n && !paths) return s3dg_internal_fail(S3DG_EINVAL, "null path list");
    for (uint64_t j = 0; j < n; ++j)
        if (!paths[j] || !paths[j][0]) return s3dg_internal_fail(S3DG_EINVAL, "empty path");
    if (object_type != S3DG_OBJ_RAW && object_type != S3DG_OBJ_TFRECORD && object_type != S3DG_OBJ_NPZ) {
        if (object_type == S3DG_OBJ_HDF5)
            return s3dg_internal_fail(S3DG_EINVAL, "HDF5 format is not available in this build");
        return s3dg_internal_fail(S3DG_EINVAL, "unknown object type");
    }
    if (payload < S3DG_PAYLOAD_CONTROLLED || payload > S3DG_PAYLOAD_DGEN)
        return s3dg_internal_fail(S3DG_EINVAL, "unknown payload kind");
    if (f_den == 0 || f_num >= f_den) return s3dg_internal_fail(S3DG_EINVAL, "need f_num < f_den");
    if (size > 0xFFFFFFFFull * kBlk) return s3dg_internal_fail(S3DG_EINVAL, "object too large");
    if (stats) *stats = s3dg_put_stats{0, 0, 0.0, 0.0};
    if (n == 0) return S3DG_OK;

    // lanes: one per context, each on its own (device, lane) pool
    const uint32_t L = (uint64_t)nctx < n ? nctx : (uint32_t)n;
    std::vector<int> devs(L);
    std::vector<PutPool *> pools(L);
    std::vector<std::unique_lock<std::mutex>> locks;
    std::map<int, int> lane_of_dev;
    for (uint32_t k = 0; k < L; ++k) {
        if (int r = s3dg_internal_ctx_device(ctxs[k], &devs[k])) return r;
        pools[k] = &pool(devs[k], lane_of_dev[devs[k]]++);
    }
    for (uint32_t k = 0; k < L; ++k) {
        locks.emplace_back(pools[k]->mu);
        DeviceScope ds(devs[k]);
        if (int r = pool_init(*pools[k], devs[k])) return r;
    }

    Writers W;
    W.outstanding.assign(L, std::array<int, kHostSlots>{});
    uint32_t nthreads = max_in_flight == 0 ? 64 : (max_in_flight > 512 ? 512 : max_in_flight);
    // file writes are memcpy into the page cache: more writers than CPUs only
    // contend (measured: 64 writers on a 16-CPU share run at half the rate of 16)
    const uint32_t cpus = usable_cpus();
    if (nthreads > cpus) nthreads = cpus;
    const uint32_t nw = (uint64_t)nthreads < n ? nthreads : (uint32_t)n;
    for (uint32_t k = 0; k < nw; ++k) W.th.emplace_back([&W] { W.run(); });

    PutArgs A{paths, n, size, object_type, payload, dedup, f_num, f_den, seed_base, crc_out, 0};
    {
        std::vector<uint8_t> pre0, suf0;
        object_frame(object_type, 1, size, 0, pre0, suf0);       // sizes of the framing
        A.pre_len = pre0.size();
    }

    int rc = S3DG_OK;
    double gpu_wait = 0.0;
    if (size == 0) {                       // framing only: no GPU work
        for (uint64_t j = 0; j < n; ++j) {
            Job job;
            job.path = paths[j];
            frame_job(A, j, 0, job);
            job.data_off = job.pre.size();
            W.push(std::move(job));
        }
    } else {
        // contiguous object ranges per lane; each lane's thread runs near its GPU
        std::vector<int> lrc(L, S3DG_OK);
        std::vector<double> lwait(L, 0.0);
        std::vector<std::string> lerr(L);
        auto lane_main = [&](uint32_t k) {
            NumaScope numa(devs[k]);
            DeviceScope ds(devs[k]);
            if (!ds.ok()) {
                lrc[k] = s3dg_internal_fail(S3DG_EHIP, "hipSetDevice");
            } else {
                const uint64_t q = n / L, r = n % L;
                const uint64_t j0 = k * q + (k < r ? k : r), j1 = j0 + q + (k < r ? 1 : 0);
                lrc[k] = run_lane(A, ctxs[k], *pools[k], (int)k, j0, j1, W, lwait[k]);
            }
            if (lrc[k] != S3DG_OK) {
                lerr[k] = s3dg_last_error();   // thread-local: carry it to the caller's thread
                W.fail(lerr[k]);
            }
        };
        if (L == 1) {
            lane_main(0);
        } else {
            std::vector<std::thread> lt;
            for (uint32_t k = 0; k < L; ++k) lt.emplace_back(lane_main, k);
            for (auto &t : lt) t.join();
        }
        for (uint32_t k = 0; k < L; ++k) {
            if (lwait[k] > gpu_wait) gpu_wait = lwait[k];
            if (rc == S3DG_OK && lrc[k] != S3DG_OK) {
                rc = lrc[k];
                s3dg_internal_fail(rc, lerr[k].c_str());
            }
        }
    }
    W.finish();
    if (rc == S3DG_OK && W.failed.load()) rc = s3dg_internal_fail(S3DG_EIO, W.err.c_str());
    if (stats) {
        stats->objects = W.files.load();
        stats->bytes = W.bytes.load();
        stats->seconds = now_s() - t0;
        stats->gpu_seconds = gpu_wait;
    }
    return rc;
}

extern "C" int s3dg_put_objects(s3dg_ctx *ctx, const char *const *paths, uint64_t n, uint64_t size,
                                int object_type, int payload, uint64_t dedup, uint32_t f_num,
                                uint32_t f_den, uint64_t seed_base, uint32_t max_in_flight,
                                uint32_t *crc_out, s3dg_put_stats *stats) {
    return s3dg_put_objects_multi(&ctx, 1, paths, n, size, object_type, payload, dedup, f_num, f_den,
                                  seed_base, max_in_flight, crc_out, stats);
}
