// s3dg_numa.cpp — host memory on the GPU's NUMA node ("a
// pinned host ring on the GPU's NUMA node").  The GPU's PCI function lists
// its local CPUs in sysfs; pinned allocations are made from a thread bound to
// those CPUs, so the kernel's default local-allocation policy places the
// pages on that node.  No libnuma: sysfs + sched affinity only.
#include "s3dg_internal.h"
#include "s3dlio_gpu.h"

#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <string>

namespace s3dg {

namespace {
std::string pci_sysfs(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return "";
    std::string id(bus);
    for (auto &ch : id) ch = (char)std::tolower((unsigned char)ch);
    return "/sys/bus/pci/devices/" + id;
}

// "0-15,64-79" -> set
bool parse_cpulist(const char *s, cpu_set_t *out) {
    CPU_ZERO(out);
    int n = 0;
    while (*s && *s != '\n') {
        char *end = nullptr;
        long a = strtol(s, &end, 10);
        if (end == s) return false;
        long b = a;
        s = end;
        if (*s == '-') {
            b = strtol(s + 1, &end, 10);
            s = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) { CPU_SET((int)c, out); ++n; }
        if (*s == ',') ++s;
    }
    return n > 0;
}
}  // namespace

bool device_local_cpus(int device, cpu_set_t *out) {
    const std::string dir = pci_sysfs(device);
    if (dir.empty()) return false;
    FILE *f = fopen((dir + "/local_cpulist").c_str(), "r");
    if (!f) return false;
    char buf[4096] = {0};
    const bool ok = fgets(buf, sizeof(buf), f) != nullptr && parse_cpulist(buf, out);
    fclose(f);
    return ok;
}

int device_numa_node(int device) {
    const std::string dir = pci_sysfs(device);
    if (dir.empty()) return -1;
    FILE *f = fopen((dir + "/numa_node").c_str(), "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}

NumaScope::NumaScope(int device) {
    cpu_set_t local, cur, both;
    if (!device_local_cpus(device, &local)) return;
    if (pthread_getaffinity_np(pthread_self(), sizeof(cur), &cur) != 0) return;
    CPU_AND(&both, &local, &cur);
    if (CPU_COUNT(&both) == 0 || CPU_EQUAL(&both, &cur)) return;   // nothing to narrow
    if (pthread_setaffinity_np(pthread_self(), sizeof(both), &both) != 0) return;
    saved_ = cur;
    active_ = true;
}

NumaScope::~NumaScope() {
    if (active_) (void)pthread_setaffinity_np(pthread_self(), sizeof(saved_), &saved_);
}

}  // namespace s3dg

using namespace s3dg;

extern "C" int s3dg_device_numa_node(int device, int *node) {
    if (!node) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    *node = device_numa_node(device);
    return S3DG_OK;
}

extern "C" int s3dg_host_alloc_pinned_local(int device, uint64_t bytes, void **out) {
    if (!out) return s3dg_internal_fail(S3DG_EINVAL, "null output");
    const hipError_t e = host_alloc_pinned_local(device, bytes, out);
    if (e != hipSuccess) return s3dg_internal_fail(S3DG_EHIP, (std::string("hipHostMalloc: ") + hipGetErrorString(e)).c_str());
    return S3DG_OK;
}
