// s3dg_host.cpp — host-buffer drop-ins on every visible GPU.
//
// The reference's host-memory entry points (fill_controlled_data,
// src/data_gen.rs:151; generate_random_data, :102; the dgen-backed
// DataGenerator / Generator / generate_data, src/data_gen.rs:253-371,
// src/python_api/python_datagen_api.rs:49-365) are synchronous, thread-safe
// and run in parallel from many threads (tests/test_s3dlio_datagen.py:174-204
// runs 8 generators at once).  Here they run on a pool of SLOTS, one per GPU
// by default:
//   * a slot = one device, its context (default base block), its copies of the
//     per-process random base blocks (A_BASE_BLOCK / BASE_BLOCK,
//     src/constants.rs:715-729) and a pool of staging sets (two 64 MiB device
//     chunks + two streams + a 4 KiB block for a caller's base block);
//   * every call takes a slot round-robin and a staging set of its own, so
//     concurrent calls never wait on a lock while the GPU works, and calls on
//     different slots use different GPUs (and PCIe links);
//   * a large call (>= 2 x kSplitMin bytes) is cut into contiguous block ranges,
//     one per slot, generated in parallel (one host thread per extra slot).
// Slot devices: S3DLIO_GPU_DEVICE=k pins every call to GPU k;
// S3DLIO_GPU_DEVICES=a,b,... lists them (repeats give several slots on one
// GPU); neither set: every visible GPU, except in one rank of a multi-process
// job (WORLD_SIZE > 1 and LOCAL_RANK set, as torch.distributed.run exports),
// which keeps to its own GPU (LOCAL_RANK mod the visible count) so ranks do not
// spread onto each other's devices.  Bytes never depend on the slot.
// D2H mode (S3DLIO_HOST_D2H): "direct" (default) copies each device chunk
// straight into the caller's buffer (hipMemcpyAsync; HIP stages pageable
// memory itself); "staged" copies into a pinned bounce buffer of the staging
// set and from there into the caller's buffer with host threads, overlapped
// with the next chunk (DESIGN.md §5.8 has the A/B).
// Registration (s3dg_host_register, explicit): a caller buffer it names is
// page-locked with hipHostRegister, and calls inside it are written by the
// kernel directly, as library-pinned memory (the criterion loop of
// benches/performance_microbenchmarks.rs:43-64 reuses one buffer).  The
// buffer must stay allocated until s3dg_host_unregister(buf) (the bindings
// hold it: s3dlio_amd.register_host_buffer, HostRegistration in the Rust
// patch).
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <sys/random.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using namespace s3dg;

namespace {

constexpr uint64_t kChunk = 64ull << 20;       // bytes per device staging chunk
constexpr uint64_t kSplitMin = 128ull << 20;   // smallest per-slot share of a split call
constexpr int kMaxSlots = 64;
// Calls that skip the copy engine (DESIGN.md §5.8 has the measurements):
// * into pinned memory this library allocated, up to kDirectMax bytes: the
//   kernel stores the caller's bytes straight into it (1 MiB 33 us against
//   42 us through the copy engine; 4 MiB 94 against 103);
// * into any other buffer, up to small_max() bytes: the kernel stores into a
//   pinned bounce buffer in pieces, and the calling thread copies piece k out
//   while pieces k+1.. are generated (64 KiB 16 us against 26, 1 MiB 55
//   against 76).  Above ~1 MiB one thread's copy out of memory the GPU has
//   just written (~30 GB/s) loses to HIP's own pageable copy path, and
//   helper threads for the copy-out measured no faster.
constexpr uint64_t kSmallMaxCap = 16ull << 20;
constexpr uint64_t kDirectMax = 16ull << 20;
constexpr uint64_t kSmallDefault = 1ull << 20;
constexpr uint64_t kPieceMin = 256ull << 10;   // smallest bounce piece
constexpr int kPiecesMax = 2;                  // pieces per small call (<= kSmallPieces; 2 and 4 measured equal)
constexpr int kMaxRings = 64;                  // read-ahead rings in existence at once

#define H_TRY(expr, what)                                                                  \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return s3dg_internal_fail(S3DG_EHIP, (std::string(what) + ": " + hipGetErrorString(e_)).c_str()); \
    } while (0)

struct Slot {
    int device = 0;
    std::mutex mu;                      // init and the idle lists
    s3dg_ctx *ctx = nullptr;            // set last: non-null = initialised
    void *base_proc[2] = {nullptr, nullptr};   // A_BASE_BLOCK, BASE_BLOCK copies in HBM
    std::vector<HostStaging *> idle;
    std::vector<HostRing *> rings;      // idle read-ahead rings
};

struct Pool {
    std::mutex mu;
    std::atomic<bool> ready{false};   // set once, under mu, after the slots exist
    std::vector<Slot *> slots;          // never freed: outlives HIP teardown
    uint8_t proc_base[2][kBlk];         // per-process random blocks (same on every slot)
    std::atomic<uint64_t> ticket{0};
    std::atomic<int> rings{0};          // read-ahead rings allocated
};

Pool &pool() {
    static Pool *p = new Pool();
    return *p;
}

int random_bytes(uint8_t *dst, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t k = getrandom(dst + got, n - got, 0);
        if (k <= 0) return s3dg_internal_fail(S3DG_EINVAL, "getrandom failed");
        got += (size_t)k;
    }
    return S3DG_OK;
}

uint64_t time_entropy() {      // SystemTime::now() ... as_nanos() as u64, src/data_gen.rs:192-195
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int pool_init(Pool &P) {
    if (P.ready.load(std::memory_order_acquire)) return S3DG_OK;   // every call after the first
    std::lock_guard<std::mutex> g(P.mu);
    if (P.ready.load(std::memory_order_relaxed)) return S3DG_OK;
    int ndev = 0;
    H_TRY(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (ndev <= 0) return s3dg_internal_fail(S3DG_EHIP, "no GPU visible");
    int devs[kMaxSlots], n = 0;
    if (int r = s3dg_host_parse_devices_env(getenv("S3DLIO_GPU_DEVICE"), getenv("S3DLIO_GPU_DEVICES"),
                                            getenv("LOCAL_RANK"), getenv("WORLD_SIZE"), ndev, devs, kMaxSlots, &n))
        return r;
    for (int k = 0; k < 2; ++k)
        if (int r = random_bytes(P.proc_base[k], kBlk)) return r;
    for (int k = 0; k < n; ++k) {
        Slot *s = new Slot();
        s->device = devs[k];
        P.slots.push_back(s);
    }
    P.ready.store(true, std::memory_order_release);
    return S3DG_OK;
}

// Context and base blocks of a slot, created under the slot's device; on any
// failure everything allocated so far is released and the slot stays
// uninitialised (the next call retries).
int slot_init(Pool &P, Slot *S) {
    std::lock_guard<std::mutex> g(S->mu);
    if (S->ctx) return S3DG_OK;
    s3dg_ctx *c = nullptr;
    if (int r = s3dg_ctx_create(S->device, &c)) return r;
    DeviceScope ds(S->device);
    void *b[2] = {nullptr, nullptr};
    hipError_t e = ds.err;
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
        e = hipMalloc(&b[k], kBlk);
        if (e == hipSuccess) e = hipMemcpy(b[k], P.proc_base[k], kBlk, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        for (void *p : b)
            if (p) (void)hipFree(p);
        s3dg_ctx_destroy(c);
        return s3dg_internal_fail(S3DG_EHIP, (std::string("host slot init: ") + hipGetErrorString(e)).c_str());
    }
    S->base_proc[0] = b[0];
    S->base_proc[1] = b[1];
    S->ctx = c;
    return S3DG_OK;
}

int get_slot(int k, Slot **out) {
    Pool &P = pool();
    if (int r = pool_init(P)) return r;
    if (k < 0 || k >= (int)P.slots.size()) return s3dg_internal_fail(S3DG_EINVAL, "host slot out of range");
    if (int r = slot_init(P, P.slots[k])) return r;
    *out = P.slots[k];
    return S3DG_OK;
}

void staging_free(HostStaging *sg) {
    for (int q = 0; q < 2; ++q) {
        if (sg->buf[q]) (void)hipFree(sg->buf[q]);
        if (sg->st[q]) (void)hipStreamDestroy(sg->st[q]);
        if (sg->pin[q]) (void)hipHostFree(sg->pin[q]);
    }
    if (sg->bounce) {
        pinned_unregister(sg->bounce);
        (void)hipHostFree(sg->bounce);
    }
    for (auto &e : sg->ev)
        if (e) (void)hipEventDestroy(e);
    if (sg->base_user) (void)hipFree(sg->base_user);
    delete sg;
}

uint64_t small_max() {
    static const uint64_t v = [] {
        const char *e = getenv("S3DLIO_HOST_SMALL_MAX");   // bytes; 0 = every call through the copy engine
        if (!e || !*e) return kSmallDefault;
        const uint64_t x = strtoull(e, nullptr, 10);
        return x < kSmallMaxCap ? x : kSmallMaxCap;
    }();
    return v;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

bool d2h_staged() {
    static const bool staged = [] {
        const char *v = getenv("S3DLIO_HOST_D2H");
        return v && strcmp(v, "staged") == 0;
    }();
    return staged;
}

// memcpy of n bytes split over up to 8 threads (>= 8 MiB per part): one host
// thread copies 10-20 GB/s, below one PCIe link.
void par_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
    constexpr uint64_t kPart = 8ull << 20;
    uint64_t parts = n / kPart;
    if (parts > 8) parts = 8;
    if (parts < 2) {
        memcpy(dst, src, n);
        return;
    }
    const uint64_t per = (n / parts + 4095) / 4096 * 4096;
    std::thread th[8];
    for (uint64_t p = 1; p < parts; ++p) {
        const uint64_t lo = p * per, hi = p + 1 == parts ? n : (p + 1) * per;
        th[p] = std::thread([=] { memcpy(dst + lo, src + lo, hi - lo); });
    }
    memcpy(dst, src, per);
    for (uint64_t p = 1; p < parts; ++p) th[p].join();
}

const void *base_for(Slot *S, HostStaging *sg, const HostJob &J) {
    switch (J.base) {
    case HostJob::kBaseProcA: return S->base_proc[0];
    case HostJob::kBaseProcB: return S->base_proc[1];
    case HostJob::kBaseUser: return sg->base_user;
    default: return ctx_base(S->ctx);
    }
}

}  // namespace

namespace s3dg {

namespace {
struct PinRegistry {
    std::mutex mu;
    std::map<uintptr_t, uint64_t> m;   // start -> bytes
};
PinRegistry &pinreg() {
    static PinRegistry *r = new PinRegistry();   // never freed: outlives static teardown
    return *r;
}
}  // namespace

void pinned_register(const void *p, uint64_t n) {
    if (!p || !n) return;
    PinRegistry &R = pinreg();
    std::lock_guard<std::mutex> g(R.mu);
    R.m[(uintptr_t)p] = n;
}

void pinned_unregister(const void *p) {
    PinRegistry &R = pinreg();
    std::lock_guard<std::mutex> g(R.mu);
    R.m.erase((uintptr_t)p);
}

bool pinned_owned(const void *p, uint64_t n) {
    const uintptr_t a = (uintptr_t)p;
    {
        PinRegistry &R = pinreg();
        std::lock_guard<std::mutex> g(R.mu);
        auto it = R.m.upper_bound(a);
        if (it == R.m.begin()) return false;
        --it;
        if (!(a >= it->first && n <= it->second && a - it->first <= it->second - n)) return false;
    }
    // and HIP still knows it as pinned host memory (a registry entry outlives a
    // buffer freed behind the library's back; a kernel must never store into
    // pageable memory: without XNACK that is a GPU page fault)
    // at both ends of the range: a registry entry whose buffer was freed and
    // whose start address a smaller pinned allocation reuses passes at p
    // alone
    auto host_pinned = [](const void *q) {
        hipPointerAttribute_t at{};
        const bool ok = hipPointerGetAttributes(&at, q) == hipSuccess && at.type == hipMemoryTypeHost;
        (void)hipGetLastError();
        return ok;
    };
    return host_pinned(p) && (n <= 1 || host_pinned((const uint8_t *)p + (n - 1)));
}

hipError_t host_alloc_pinned_local(int device, uint64_t bytes, void **out) {
    *out = nullptr;
    DeviceScope ds(device);
    if (!ds.ok()) return ds.err;
    NumaScope scope(device);
    const hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
    if (e == hipSuccess) pinned_register(*out, bytes);
    return e;
}

int host_slot_count(int *n) {
    Pool &P = pool();
    if (int r = pool_init(P)) return r;
    *n = (int)P.slots.size();
    return S3DG_OK;
}

int host_next_slot(int *slot) {
    int n = 0;
    if (int r = host_slot_count(&n)) return r;
    *slot = (int)(pool().ticket.fetch_add(1) % (uint64_t)n);
    return S3DG_OK;
}

int host_staging_acquire(int slot, HostStaging **out) {
    Slot *S = nullptr;
    if (int r = get_slot(slot, &S)) return r;
    {
        std::lock_guard<std::mutex> g(S->mu);
        if (!S->idle.empty()) {
            *out = S->idle.back();
            S->idle.pop_back();
            return S3DG_OK;
        }
    }
    DeviceScope ds(S->device);
    HostStaging *sg = new HostStaging();
    sg->slot = slot;
    hipError_t e = ds.err;
    for (int q = 0; q < 2 && e == hipSuccess; ++q) {
        e = hipMalloc(&sg->buf[q], kChunk);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&sg->st[q], hipStreamNonBlocking);
    }
    if (e == hipSuccess) e = hipMalloc(&sg->base_user, kBlk);
    if (e != hipSuccess) {
        staging_free(sg);
        return s3dg_internal_fail(S3DG_EHIP, (std::string("host staging: ") + hipGetErrorString(e)).c_str());
    }
    *out = sg;
    return S3DG_OK;
}

void host_staging_release(HostStaging *sg) {
    if (!sg) return;
    Slot *S = pool().slots[sg->slot];
    {
        // every caller has normally drained the streams already (a call
        // returns after its last copy); a query costs less than a synchronize
        DeviceScope ds(S->device);
        for (int q = 0; q < 2; ++q)
            if (hipStreamQuery(sg->st[q]) != hipSuccess) (void)hipStreamSynchronize(sg->st[q]);
        (void)hipGetLastError();
    }
    std::lock_guard<std::mutex> g(S->mu);
    S->idle.push_back(sg);
}

int host_ring_acquire(int slot, uint64_t half, HostRing **out) {
    *out = nullptr;
    Slot *S = nullptr;
    if (int r = get_slot(slot, &S)) return r;
    {
        std::lock_guard<std::mutex> g(S->mu);
        for (size_t k = 0; k < S->rings.size(); ++k)
            if (S->rings[k]->half == half) {
                *out = S->rings[k];
                S->rings.erase(S->rings.begin() + (long)k);
                return S3DG_OK;
            }
    }
    Pool &P = pool();
    if (P.rings.fetch_add(1) >= kMaxRings) {   // enough pinned rings: this generator runs synchronously
        P.rings.fetch_sub(1);
        return S3DG_OK;
    }
    HostRing *r = new HostRing();
    r->slot = slot;
    r->half = half;
    void *mem = nullptr;
    hipError_t e = host_alloc_pinned_local(S->device, 2 * half, &mem);
    DeviceScope ds(S->device);
    for (int q = 0; q < 2 && e == hipSuccess; ++q) e = hipEventCreateWithFlags(&r->ev[q], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (auto &ev : r->ev)
            if (ev) (void)hipEventDestroy(ev);
        if (mem) {
            pinned_unregister(mem);
            (void)hipHostFree(mem);
        }
        delete r;
        P.rings.fetch_sub(1);
        return s3dg_internal_fail(S3DG_EHIP, (std::string("read-ahead ring: ") + hipGetErrorString(e)).c_str());
    }
    r->mem = (uint8_t *)mem;
    *out = r;
    return S3DG_OK;
}

void host_ring_release(HostRing *r) {
    if (!r) return;
    Slot *S = pool().slots[r->slot];
    std::lock_guard<std::mutex> g(S->mu);
    S->rings.push_back(r);
}

// Bytes [pos, pos+n) of the job's object into host `buf` on the staging set's
// slot: the covering generation blocks go through the two device chunks on
// two streams (chunk k+1's kernel overlaps chunk k's D2H), then exactly the
// requested bytes are copied out (directly, or through the pinned bounce
// buffers in staged mode, where chunk k's host copy overlaps chunk k+1's
// kernel and D2H).  On an error the streams are drained before returning, so
// no copy is still landing in `buf` when the caller sees the failure.
// The caller's base block into the staging set's device block, unless it is
// the block uploaded last (a seeded caller passes the same block every call).
static int upload_user_base(HostStaging *sg, const HostJob &J) {
    if (J.base != HostJob::kBaseUser) return S3DG_OK;
    if (sg->base_user_valid && memcmp(sg->base_user_host, J.user_base, kBlk) == 0) return S3DG_OK;
    sg->base_user_valid = false;
    H_TRY(hipMemcpy(sg->base_user, J.user_base, kBlk, hipMemcpyHostToDevice), "hipMemcpy(base block)");
    memcpy(sg->base_user_host, J.user_base, kBlk);
    sg->base_user_valid = true;
    return S3DG_OK;
}

int host_launch_blocks(HostStaging *sg, const HostJob &J, uint8_t *dst, uint64_t b_lo, uint64_t b_hi,
                       hipStream_t st) {
    Slot *S = pool().slots[sg->slot];
    if (J.dgen)
        return s3dg_dgen_fill(S->ctx, dst, J.obj_len, b_lo, b_hi, J.dedup, J.f_num, J.f_den, J.entropy, st);
    H_TRY(launch_fill_stream(ctx_stream_cfg(S->ctx), dst, J.obj_len, 0, 1, (uint32_t)b_lo, (uint32_t)b_hi,
                             J.entropy, 0, J.pp, base_for(S, sg, J), st),
          "launch k_fill_stream(host)");
    return S3DG_OK;
}

// ---- explicit registration of caller buffers (s3dg_host_register)
//
// Round 5 registered a pageable buffer on its second sighting (env
// S3DLIO_HOST_REGISTER=1).  That was unsound: a caller that frees a buffer
// never learns that it was registered, and a buffer freed and re-mapped at the
// same address kept the registration.  On
// ROCm the driver drops a registered range's GPU mapping when its pages are
// unmapped, so the next kernel store into it is a GPU memory fault (measured
// round 6: munmap + mmap(MAP_FIXED) + a call = "illegal memory access"); no
// check the host can make before a launch sees that.  So a buffer is
// registered only by the caller's own call, with hipHostRegister's contract:
// it stays allocated until s3dg_host_unregister.  The bindings enforce that
// lifetime: the Python handle holds an export of the buffer (it cannot be
// freed while registered), the Rust guard borrows the slice.
namespace {
struct UserReg {
    uint64_t bytes;    // page-rounded length
    uint8_t *dev;      // device pointer of the first page
    int users;         // host calls in flight on it (they hold it until they return)
};
struct UserRegs {
    std::mutex mu;
    std::condition_variable cv;                      // a registration's users dropped to 0
    std::map<uintptr_t, UserReg> regs;               // page start -> registration
};
UserRegs &userregs() {
    static UserRegs *r = new UserRegs();   // never freed: outlives static teardown
    return *r;
}

// Unregisters every registration matching `hit` once no call uses it (R.mu
// held through `g`, released while waiting).  Returns how many it dropped.
template <class Hit>
int drop_regs(UserRegs &R, std::unique_lock<std::mutex> &g, Hit hit) {
    int dropped = 0;
    for (;;) {
        bool busy = false;
        for (auto q = R.regs.begin(); q != R.regs.end();) {
            if (!hit(q->first, q->second.bytes)) {
                ++q;
            } else if (q->second.users > 0) {
                busy = true;
                ++q;
            } else {
                (void)hipHostUnregister((void *)q->first);
                (void)hipGetLastError();
                q = R.regs.erase(q);
                ++dropped;
            }
        }
        if (!busy) return dropped;
        R.cv.wait(g);   // another thread's call is writing into one of them
    }
}

// A host call's hold on a registered range (UserHold::key != 0), released
// when the call returns (or earlier, by release()).
struct UserHold {
    uintptr_t key = 0;
    void release() {
        if (!key) return;
        UserRegs &R = userregs();
        std::lock_guard<std::mutex> g(R.mu);
        auto it = R.regs.find(key);
        if (it != R.regs.end() && --it->second.users == 0) R.cv.notify_all();
        key = 0;
    }
    ~UserHold() { release(); }
};

// The device pointer of [p, p+n) when it lies inside a registered range; the
// call then holds that range (hold) until it returns, so no other thread
// unregisters pages it is writing.  A range that overlaps registered ones
// without lying inside one unregisters them first, once their holders have
// returned: HIP treats a copy into a partly registered range as pinned and
// fails (two buffers can share a page).  nullptr: use the regular paths.
uint8_t *user_registered(const uint8_t *p, uint64_t n, bool direct_ok, UserHold &hold) {
    UserRegs &R = userregs();
    const uintptr_t a = (uintptr_t)p;
    std::unique_lock<std::mutex> g(R.mu);
    if (R.regs.empty()) return nullptr;
    auto it = R.regs.upper_bound(a);
    if (it != R.regs.begin()) {
        --it;
        if (a >= it->first && a + n <= it->first + it->second.bytes) {
            // inside: held until the call returns, direct or not (a copy-engine
            // copy into it must not see the pages unregistered mid-flight)
            ++it->second.users;
            hold.key = it->first;
            return direct_ok ? it->second.dev + (a - it->first) : nullptr;
        }
    }
    const uintptr_t lo = a & ~(uintptr_t)4095, hi = (a + n + 4095) & ~(uintptr_t)4095;
    drop_regs(R, g, [&](uintptr_t s0, uint64_t len) { return s0 < hi && s0 + len > lo; });
    return nullptr;
}

}  // namespace

extern "C" int s3dg_host_register(void *buf, uint64_t len) {
    if (!buf || len == 0) return s3dg_internal_fail(S3DG_EINVAL, "s3dg_host_register: null buffer or zero length");
    UserRegs &R = userregs();
    const uintptr_t a = (uintptr_t)buf;
    const uintptr_t lo = a & ~(uintptr_t)4095, hi = (a + len + 4095) & ~(uintptr_t)4095;
    std::unique_lock<std::mutex> g(R.mu);
    auto it = R.regs.find(lo);
    if (it != R.regs.end() && it->second.bytes == hi - lo) return S3DG_OK;   // already registered
    drop_regs(R, g, [&](uintptr_t s0, uint64_t l) { return s0 < hi && s0 + l > lo; });
    hipError_t e = hipHostRegister((void *)lo, hi - lo, hipHostRegisterPortable | hipHostRegisterMapped);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return s3dg_internal_fail(S3DG_EHIP, (std::string("hipHostRegister: ") + hipGetErrorString(e)).c_str());
    }
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, (void *)lo, 0);
    if (e != hipSuccess || !d) {
        (void)hipGetLastError();
        (void)hipHostUnregister((void *)lo);
        (void)hipGetLastError();
        return s3dg_internal_fail(S3DG_EHIP, "hipHostGetDevicePointer failed for a registered buffer");
    }
    R.regs[lo] = UserReg{hi - lo, (uint8_t *)d, 0};
    return S3DG_OK;
}

extern "C" int s3dg_host_unregister(void *buf) {
    UserRegs &R = userregs();
    std::unique_lock<std::mutex> g(R.mu);
    const uintptr_t a = (uintptr_t)buf;
    // waits for calls still writing into a matching range (other threads')
    return drop_regs(R, g, [&](uintptr_t s0, uint64_t len) { return !buf || (a >= s0 && a < s0 + len); });
}

// The kernel may write the request's covering blocks straight into `buf`:
// pinned memory this library allocated, 16-B aligned, and the blocks start
// and end exactly at the request.
static bool direct_geometry(const HostJob &J, const uint8_t *buf, uint64_t pos, uint64_t n) {
    const uint64_t unit = J.dgen ? kDgenBlock : kBlk;
    return n <= kDirectMax && aligned16(buf) && pos % unit == 0 && ((pos + n) % unit == 0 || pos + n == J.obj_len);
}

static bool direct_target(const HostJob &J, const uint8_t *buf, uint64_t pos, uint64_t n) {
    return direct_geometry(J, buf, pos, n) && pinned_owned(buf, n);
}

// A call without the copy engine: straight into the caller's buffer
// (direct_target), or through the staging set's pinned bounce buffer in up
// to kPiecesMax pieces on one stream, the calling thread copying piece k out
// while pieces k+1.. are generated.
// kdst: the device-visible address of buf (registered user memory), or buf.
static int host_run_small(HostStaging *sg, Slot *S, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n,
                          bool direct, uint8_t *kdst) {
    if (int r = upload_user_base(sg, J)) return r;
    const uint64_t unit = J.dgen ? kDgenBlock : kBlk;
    const uint64_t b0 = pos / unit, b1 = (pos + n + unit - 1) / unit;
    hipStream_t st = sg->st[0];
    if (direct) {
        if (int r = host_launch_blocks(sg, J, kdst, b0, b1, st)) return r;
        H_TRY(hipStreamSynchronize(st), "hipStreamSynchronize");
        return S3DG_OK;
    }
    const uint64_t need = small_max() + 2 * kDgenBlock;   // the covering blocks of any small request
    if (sg->bounce_bytes < need) {
        if (sg->bounce) {
            pinned_unregister(sg->bounce);
            H_TRY(hipHostFree(sg->bounce), "hipHostFree(bounce)");
            sg->bounce = nullptr;
            sg->bounce_bytes = 0;
        }
        void *p = nullptr;
        H_TRY(host_alloc_pinned_local(S->device, need, &p), "hipHostMalloc(bounce)");
        sg->bounce = (uint8_t *)p;
        sg->bounce_bytes = need;
    }
    const uint64_t nb = b1 - b0;
    const uint64_t min_per = (kPieceMin + unit - 1) / unit;
    uint64_t per = (nb + kPiecesMax - 1) / kPiecesMax;
    if (per < min_per) per = min_per;
    const int np = (int)((nb + per - 1) / per);
    for (int k = 0; k < np; ++k) {
        if (!sg->ev[k]) H_TRY(hipEventCreateWithFlags(&sg->ev[k], hipEventDisableTiming), "hipEventCreate");
        const uint64_t pb = b0 + k * per, pe = pb + per < b1 ? pb + per : b1;
        if (int r = host_launch_blocks(sg, J, sg->bounce + (pb - b0) * unit, pb, pe, st)) return r;
        H_TRY(hipEventRecord(sg->ev[k], st), "hipEventRecord");
    }
    for (int k = 0; k < np; ++k) {
        const uint64_t pb = b0 + k * per, pe = pb + per < b1 ? pb + per : b1;
        H_TRY(hipEventSynchronize(sg->ev[k]), "hipEventSynchronize");
        const uint64_t lo = pb * unit > pos ? pb * unit : pos;
        const uint64_t hi = pe * unit < pos + n ? pe * unit : pos + n;
        if (hi > lo) memcpy(buf + (lo - pos), sg->bounce + (lo - b0 * unit), hi - lo);
    }
    return S3DG_OK;
}

static int host_run_chunks(HostStaging *sg, Slot *S, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (int r = upload_user_base(sg, J)) return r;
    const void *base = base_for(S, sg, J);
    const bool staged = d2h_staged();
    if (staged)
        for (int q = 0; q < 2; ++q)
            if (!sg->pin[q]) H_TRY(hipHostMalloc(&sg->pin[q], kChunk, hipHostMallocDefault), "hipHostMalloc(bounce)");
    const uint64_t unit = J.dgen ? kDgenBlock : kBlk;
    const uint64_t per = kChunk / unit;
    const uint64_t b0 = pos / unit, b1 = (pos + n + unit - 1) / unit;
    uint64_t pend_lo[2] = {0, 0}, pend_len[2] = {0, 0};   // staged: copied-out ranges per bounce buffer
    auto drain = [&](int sl) -> int {                      // staged: bounce buffer sl -> buf
        if (!pend_len[sl]) return S3DG_OK;
        H_TRY(hipStreamSynchronize(sg->st[sl]), "hipStreamSynchronize");
        par_copy(buf + (pend_lo[sl] - pos), (const uint8_t *)sg->pin[sl], pend_len[sl]);
        pend_len[sl] = 0;
        return S3DG_OK;
    };
    int k = 0;
    for (uint64_t pb = b0; pb < b1; pb += per, ++k) {
        const uint64_t pe = pb + per < b1 ? pb + per : b1;
        const int sl = k & 1;
        if (J.dgen) {
            if (int r = s3dg_dgen_fill(S->ctx, sg->buf[sl], J.obj_len, pb, pe, J.dedup, J.f_num, J.f_den, J.entropy,
                                       sg->st[sl]))
                return r;
        } else {
            H_TRY(launch_fill_stream(ctx_stream_cfg(S->ctx), (uint8_t *)sg->buf[sl], J.obj_len, 0, 1, (uint32_t)pb,
                                     (uint32_t)pe, J.entropy, 0, J.pp, base, sg->st[sl]),
                  "launch k_fill_stream(host chunk)");
        }
        const uint64_t lo = pb * unit > pos ? pb * unit : pos;
        const uint64_t hi = pe * unit < pos + n ? pe * unit : pos + n;
        const uint8_t *src = (uint8_t *)sg->buf[sl] + (lo - pb * unit);
        if (staged) {
            H_TRY(hipMemcpyAsync(sg->pin[sl], src, hi - lo, hipMemcpyDeviceToHost, sg->st[sl]), "hipMemcpyAsync(D2H)");
            pend_lo[sl] = lo;
            pend_len[sl] = hi - lo;
            if (int r = drain(sl ^ 1)) return r;          // chunk k-1, while chunk k runs
        } else {
            H_TRY(hipMemcpyAsync(buf + (lo - pos), src, hi - lo, hipMemcpyDeviceToHost, sg->st[sl]),
                  "hipMemcpyAsync(D2H)");
        }
    }
    if (staged) {
        for (int q = 0; q < 2; ++q)
            if (int r = drain((k + q) & 1)) return r;     // oldest first
    }
    H_TRY(hipStreamSynchronize(sg->st[0]), "hipStreamSynchronize");
    H_TRY(hipStreamSynchronize(sg->st[1]), "hipStreamSynchronize");
    return S3DG_OK;
}

int host_run(HostStaging *sg, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n) {
    if (n == 0) return S3DG_OK;
    Slot *S = pool().slots[sg->slot];
    DeviceScope ds(S->device);
    H_TRY(ds.err, "hipSetDevice");
    bool direct = !d2h_staged() && direct_target(J, buf, pos, n);
    uint8_t *kdst = buf;
    UserHold hold;   // released on return: the call's copies and kernels are done by then
    if (!direct) {
        const bool geo = !d2h_staged() && direct_geometry(J, buf, pos, n);
        if (uint8_t *d = user_registered(buf, n, geo, hold)) {   // inside a caller-registered buffer
            direct = true;
            kdst = d;
        }
    }
    const int r = direct || (n <= small_max() && !d2h_staged()) ? host_run_small(sg, S, J, buf, pos, n, direct, kdst)
                                                                : host_run_chunks(sg, S, J, buf, pos, n);
    if (r != S3DG_OK)
        for (int q = 0; q < 2; ++q) (void)hipStreamSynchronize(sg->st[q]);   // nothing lands later
    return r;
}

// The same, cut into one contiguous range per slot when the request is large
// enough: part 0 runs on `sg0` (the caller's staging, on slot sg0->slot) in
// the calling thread, part p on slot (sg0->slot + p) mod slots in a thread of
// its own with a staging set of its own.
int host_run_split(HostStaging *sg0, const HostJob &J, uint8_t *buf, uint64_t pos, uint64_t n) {
    int nslots = 1;
    if (int r = host_slot_count(&nslots)) return r;
    const uint64_t unit = J.dgen ? kDgenBlock : kBlk;
    uint64_t parts = n / kSplitMin;
    if (parts > (uint64_t)nslots) parts = (uint64_t)nslots;
    if (parts < 2) return host_run(sg0, J, buf, pos, n);
    // part boundaries on generation-block edges
    std::vector<uint64_t> cut(parts + 1);
    cut[0] = pos;
    cut[parts] = pos + n;
    for (uint64_t p = 1; p < parts; ++p) {
        uint64_t c = pos + n / parts * p;
        c = c / unit * unit;
        cut[p] = c < cut[p - 1] ? cut[p - 1] : c;
    }
    std::vector<int> rc(parts, S3DG_OK);
    std::vector<std::string> err(parts);
    std::vector<std::thread> th;
    for (uint64_t p = 1; p < parts; ++p) {
        th.emplace_back([&, p]() {
            HostStaging *sg = nullptr;
            int r = host_staging_acquire((int)((sg0->slot + p) % (uint64_t)nslots), &sg);
            if (r == S3DG_OK) r = host_run(sg, J, buf + (cut[p] - pos), cut[p], cut[p + 1] - cut[p]);
            if (r != S3DG_OK) err[p] = s3dg_last_error();
            host_staging_release(sg);
            rc[p] = r;
        });
    }
    rc[0] = host_run(sg0, J, buf, cut[0], cut[1] - cut[0]);
    for (auto &t : th) t.join();
    for (uint64_t p = 1; p < parts; ++p)
        if (rc[p] != S3DG_OK && rc[0] == S3DG_OK) return s3dg_internal_fail(rc[p], err[p].c_str());
    return rc[0];
}

// One-shot: a slot round-robin, a staging set for the call, split over slots.
static int host_oneshot(const HostJob &J, uint8_t *buf, uint64_t len) {
    int slot = 0;
    if (int r = host_next_slot(&slot)) return r;
    HostStaging *sg = nullptr;
    if (int r = host_staging_acquire(slot, &sg)) return r;
    const int r = host_run_split(sg, J, buf, 0, len);
    host_staging_release(sg);
    return r;
}

static int controlled_job(HostJob &J, uint64_t len, uint64_t dedup, uint64_t compress) {
    uint32_t fn, fd;
    if (int r = s3dg_compress_ratio(compress, &fn, &fd)) return r;
    J.obj_len = len;
    return make_prefix((len + kBlk - 1) / kBlk, dedup, fn, fd, &J.pp);
}

}  // namespace s3dg

extern "C" {

int s3dg_host_parse_devices(const char *pin, const char *list, int ndev, int *out, int cap, int *n) {
    return s3dg_host_parse_devices_env(pin, list, nullptr, nullptr, ndev, out, cap, n);
}

int s3dg_host_parse_devices_env(const char *pin, const char *list, const char *local_rank, const char *world_size,
                                int ndev, int *out, int cap, int *n) {
    if (!out || !n || cap <= 0) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *n = 0;
    auto parse_int = [&](const char *&p, int *v) -> bool {
        while (*p == ' ') ++p;
        if (*p < '0' || *p > '9') return false;
        long x = 0;
        while (*p >= '0' && *p <= '9') {
            x = x * 10 + (*p++ - '0');
            if (x > 1000000) return false;
        }
        while (*p == ' ') ++p;
        *v = (int)x;
        return true;
    };
    if (pin && *pin) {
        const char *p = pin;
        int d = 0;
        if (!parse_int(p, &d) || *p) return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICE must be a device index");
        if (d >= ndev) return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICE out of range");
        out[0] = d;
        *n = 1;
        return S3DG_OK;
    }
    if (list && *list) {
        const char *p = list;
        int k = 0;
        for (;;) {
            int d = 0;
            if (!parse_int(p, &d)) return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICES must be a comma list of device indices");
            if (d >= ndev) return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICES names a device out of range");
            if (k >= cap) return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICES lists too many slots");
            out[k++] = d;
            if (!*p) break;
            if (*p++ != ',') return s3dg_internal_fail(S3DG_EINVAL, "S3DLIO_GPU_DEVICES must be a comma list of device indices");
        }
        *n = k;
        return S3DG_OK;
    }
    if (ndev <= 0) return s3dg_internal_fail(S3DG_EINVAL, "no GPU visible");
    // one rank of a multi-process job: its own GPU only
    int ws = 0, lr = 0;
    const char *pw = world_size, *pr = local_rank;
    if (pw && *pw && pr && *pr && parse_int(pw, &ws) && !*pw && ws > 1 && parse_int(pr, &lr) && !*pr) {
        out[0] = lr % ndev;
        *n = 1;
        return S3DG_OK;
    }
    for (int d = 0; d < ndev && d < cap; ++d) out[(*n)++] = d;
    return S3DG_OK;
}

int s3dg_host_slot_count(int *out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    return host_slot_count(out);
}

int s3dg_host_slot_device(int slot, int *device) {
    if (!device) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    Pool &P = pool();
    if (int r = pool_init(P)) return r;
    if (slot < 0 || slot >= (int)P.slots.size()) return s3dg_internal_fail(S3DG_EINVAL, "host slot out of range");
    *device = P.slots[slot]->device;
    return S3DG_OK;
}

int s3dg_host_slot_context(int slot, s3dg_ctx **out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *out = nullptr;
    if (slot < 0) {
        if (int r = host_next_slot(&slot)) return r;
    }
    Slot *S = nullptr;
    if (int r = get_slot(slot, &S)) return r;
    *out = S->ctx;
    return S3DG_OK;
}

// generate_random_data payload for generate_object: seeded (the slot
// context's default base block, entropy = seed) or unseeded (time entropy +
// the per-process BASE_BLOCK).
int s3dg_internal_random_host(uint8_t *buf, uint64_t len, uint64_t entropy, int use_process_base) {
    if (len == 0) return S3DG_OK;
    const uint64_t nb = (len + kBlk - 1) / kBlk;
    if (nb > 0xFFFFFFFFull) return s3dg_internal_fail(S3DG_EINVAL, "object larger than 2^32 blocks");
    HostJob J;
    J.obj_len = len;
    J.pp = random_layout_prefix();
    J.entropy = use_process_base ? time_entropy() : entropy;
    J.base = use_process_base ? HostJob::kBaseProcB : HostJob::kBaseCtx;
    return host_oneshot(J, buf, len);
}

int s3dlio_generate_random_data(uint8_t *buf, size_t size) {
    if (size == 0) return S3DG_OK;
    if (!buf) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    return s3dg_internal_random_host(buf, size, 0, 1);
}

int s3dlio_fill_controlled_data(uint8_t *buf, size_t len, size_t dedup, size_t compress) {
    if (len == 0) return S3DG_OK;                                    // :154-156
    if (!buf) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    HostJob J;
    if (int r = controlled_job(J, len, dedup, compress)) return r;
    J.entropy = time_entropy();
    J.base = HostJob::kBaseProcA;
    return host_oneshot(J, buf, len);
}

int s3dlio_fill_controlled_data_seeded(uint8_t *buf, size_t len, size_t dedup, size_t compress,
                                       uint64_t entropy, const uint8_t *base4096) {
    if (len == 0) return S3DG_OK;
    if (!buf) return s3dg_internal_fail(S3DG_EINVAL, "null buffer");
    HostJob J;
    if (int r = controlled_job(J, len, dedup, compress)) return r;
    J.entropy = entropy;
    J.base = base4096 ? HostJob::kBaseUser : HostJob::kBaseCtx;
    J.user_base = base4096;
    return host_oneshot(J, buf, len);
}

}  // extern "C"
