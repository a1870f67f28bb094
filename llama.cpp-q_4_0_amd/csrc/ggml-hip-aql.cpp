// ggml-hip-aql.cpp — launch mode 3 of the hook path's launch recorder (GGML_HIP_GRAPH=3, ggml_hip_debug_set_graph(3)):
// every kernel goes straight into an own HSA AQL queue on the device: 0.20-0.28 us of host time per dispatch against
// 2.5-3.3 us for hipLaunchKernel (tools/aql_dispatch_cost.hip, profiles/r06_aql_dispatch_cost.txt).  The kernargs
// live in a VRAM ring written through the large-BAR mapping (in host memory the device side ran ~8x slower; in VRAM
// it equals HIP's), the kernel objects come from the code objects HIP loaded (HSA loader extension, by the kernel's
// name).  Ordering with the HIP stream the backend also uses (copies, memsets): the first dispatch after any HIP
// work waits for that stream on the host, and every backend HIP call drains the queue first (rec_flush through
// GHIP_SYNC: a barrier packet with a completion signal, waited for on the host).  A kernel this path cannot take
// (no code-object symbol, an argument layout it does not know) runs through hipLaunchKernel in order.  The hidden
// arguments filled are the dispatch geometry and the dynamic LDS size; the runtime-service pointers (hostcall /
// printf buffer, device heap, multigrid sync) stay zero, so a kernel using device printf, malloc or assert must not
// take this path (the library has none: tests/test_abi.py checks the sources).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>
#include <immintrin.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>

#include "launch.h"

namespace ghip {

namespace {

struct AqlKernel {
    uint64_t kobj = 0;
    uint32_t ksize = 0, grp = 0, prv = 0;
    bool ok = false;
    int tries = 0;                        // a symbol not found yet (code object not loaded) is looked up again
};

struct Aql {
    bool tried = false, ok = false;
    int device = -1;
    hsa_agent_t gpu{}, cpu{};
    hsa_queue_t *q = nullptr;
    char *karg = nullptr;                 // VRAM, SLOT bytes per queue entry
    hsa_signal_t done{};
    hsa_ven_amd_loader_1_03_pfn_t loader{};
    std::unordered_map<const void *, AqlKernel> kernels;
    uint64_t submitted = 0;               // dispatches since the last drain
    bool stream_dirty = true;             // HIP work may be pending on the backend stream
    long long dispatches = 0, fallbacks = 0, drains = 0, stream_syncs = 0;
};
constexpr size_t SLOT = 1024;

Aql &aql() {
    static Aql a;
    return a;
}

struct Find {
    int domain, bdf;
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
};
hsa_status_t find_agents(hsa_agent_t agent, void *data) {
    Find &f = *(Find *)data;
    hsa_device_type_t t;
    if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f.have_cpu) {
        f.cpu = agent;
        f.have_cpu = true;
    }
    if (t == HSA_DEVICE_TYPE_GPU && !f.have_gpu) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if ((int)bdf == f.bdf && (int)dom == f.domain) {
            f.gpu = agent;
            f.have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}
struct PoolFind {
    hsa_amd_memory_pool_t pool{};
    bool have = false;
};
hsa_status_t find_vram(hsa_amd_memory_pool_t pool, void *data) {
    PoolFind &p = *(PoolFind *)data;
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !p.have) {
        p.pool = pool;
        p.have = true;
    }
    return HSA_STATUS_SUCCESS;
}

bool init(Aql &a) {
    a.tried = true;
    int dev = 0, dom = 0, bus = 0, did = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess ||
        hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
        hipDeviceGetAttribute(&did, hipDeviceAttributePciDeviceId, dev) != hipSuccess)
        return false;
    if (hsa_init() != HSA_STATUS_SUCCESS) return false;
    Find f{dom, (bus << 8) | (did << 3)};
    if (hsa_iterate_agents(find_agents, &f) != HSA_STATUS_SUCCESS || !f.have_gpu || !f.have_cpu) return false;
    a.gpu = f.gpu;
    a.cpu = f.cpu;
    a.device = dev;
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(a.loader), &a.loader) != HSA_STATUS_SUCCESS)
        return false;
    if (hsa_queue_create(a.gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &a.q) != HSA_STATUS_SUCCESS)
        return false;
    PoolFind p;
    bool ok = hsa_amd_agent_iterate_memory_pools(a.gpu, find_vram, &p) == HSA_STATUS_SUCCESS && p.have &&
              hsa_amd_memory_pool_allocate(p.pool, SLOT * a.q->size, 0, (void **)&a.karg) == HSA_STATUS_SUCCESS;
    ok = ok && hsa_amd_agents_allow_access(1, &a.cpu, nullptr, a.karg) == HSA_STATUS_SUCCESS;
    ok = ok && hsa_signal_create(1, 0, nullptr, &a.done) == HSA_STATUS_SUCCESS;
    if (!ok) {                            // a partial set-up is released: this process then launches through HIP
        if (a.karg) (void)hsa_amd_memory_pool_free(a.karg);
        a.karg = nullptr;
        (void)hsa_queue_destroy(a.q);
        a.q = nullptr;
    }
    return ok;
}

struct SymFind {
    const char *name;
    hsa_agent_t gpu;
    hsa_executable_symbol_t sym{};
    bool have = false;
};
hsa_status_t find_symbol(hsa_executable_t exe, void *data) {
    SymFind &s = *(SymFind *)data;
    if (s.have) return HSA_STATUS_SUCCESS;
    hsa_executable_symbol_t sym;
    if (hsa_executable_get_symbol_by_name(exe, s.name, &s.gpu, &sym) == HSA_STATUS_SUCCESS) {
        s.sym = sym;
        s.have = true;
    }
    return HSA_STATUS_SUCCESS;
}

const AqlKernel &kernel_of(Aql &a, const void *fn, hipStream_t s) {
    auto it = a.kernels.find(fn);
    if (it != a.kernels.end() && (it->second.ok || it->second.tries >= 3)) return it->second;
    AqlKernel k;
    k.tries = it != a.kernels.end() ? it->second.tries + 1 : 1;
    const char *name = hipKernelNameRefByPtr(fn, s);
    (void)hipGetLastError();
    if (name) {
        const std::string kd = std::string(name) + ".kd";
        SymFind sf{kd.c_str(), a.gpu};
        if (a.loader.hsa_ven_amd_loader_iterate_executables) a.loader.hsa_ven_amd_loader_iterate_executables(find_symbol, &sf);
        if (sf.have &&
            hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.kobj) == HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.ksize) == HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.grp) == HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.prv) == HSA_STATUS_SUCCESS)
            k.ok = k.kobj != 0 && k.ksize <= SLOT && k.prv == 0;     // no scratch: that needs the queue's scratch setup
    }
    AqlKernel &slot = a.kernels[fn];
    slot = k;
    return slot;
}

}  // namespace

bool aql_pending() { return aql().submitted > 0; }

void aql_stream_dirty() { aql().stream_dirty = true; }

void aql_counts(long long *out) {
    out[0] = aql().dispatches;
    out[1] = aql().fallbacks;
    out[2] = aql().drains;
    out[3] = aql().stream_syncs;
}

// every dispatch so far complete (a barrier-AND packet with the completion signal, waited for on the host)
void aql_drain() {
    Aql &a = aql();
    if (!a.submitted) return;
    const uint64_t idx = hsa_queue_add_write_index_relaxed(a.q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(a.q) >= a.q->size) {}
    hsa_barrier_and_packet_t *p = (hsa_barrier_and_packet_t *)a.q->base_address + (idx & (a.q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->completion_signal = a.done;
    hsa_signal_store_relaxed(a.done, 1);
    const uint16_t header = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n((uint32_t *)p, (uint32_t)header, __ATOMIC_RELEASE);
    hsa_signal_store_screlease(a.q->doorbell_signal, idx);
    // 20 s: a device that never finishes is a fault, not a wait
    if (hsa_signal_wait_scacquire(a.done, HSA_SIGNAL_CONDITION_LT, 1, 20ull * 1000000000ull, HSA_WAIT_STATE_ACTIVE) != 0) {
        fprintf(stderr, "ggml-hip: AQL launch mode: the queue did not drain\n");
        abort();
    }
    a.submitted = 0;
    a.drains++;
}

// false: this launch cannot go through the queue (the caller launches it through HIP, in order)
bool aql_dispatch(const void *fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, int nargs, void *const *args,
                  const size_t *sizes, const size_t *aligns) {
    Aql &a = aql();
    if (!a.tried) a.ok = init(a);
    int dev = -1;
    if (!a.ok || hipGetDevice(&dev) != hipSuccess || dev != a.device) return false;
    const AqlKernel &k = kernel_of(a, fn, s);
    if (!k.ok) return false;
    // explicit arguments packed as the kernel ABI lays them out (each at its alignment), then the code object v5
    // hidden block (block counts, group sizes, remainders, grid dims, dynamic LDS) when the segment has one
    alignas(16) unsigned char buf[SLOT];
    memset(buf, 0, sizeof buf);
    size_t used = 0;
    for (int i = 0; i < nargs; i++) {
        const size_t off = (used + aligns[i] - 1) & ~(aligns[i] - 1);
        if (off + sizes[i] > SLOT) return false;
        memcpy(buf + off, args[i], sizes[i]);
        used = off + sizes[i];
    }
    const size_t e = (used + 7) & ~(size_t)7;
    if (k.ksize != e && k.ksize != used) {
        if (k.ksize < e + 128) return false;                  // not the layout below
        uint32_t *u32 = (uint32_t *)(buf + e);
        uint16_t *u16 = (uint16_t *)(buf + e);
        u32[0] = grid.x;
        u32[1] = grid.y;
        u32[2] = grid.z;
        u16[6] = (uint16_t)block.x;
        u16[7] = (uint16_t)block.y;
        u16[8] = (uint16_t)block.z;
        u16[32] = (uint16_t)(grid.z > 1 || block.z > 1 ? 3 : grid.y > 1 || block.y > 1 ? 2 : 1);   // +64: grid dims
        u32[30] = (uint32_t)lds;                                                                       // +120
    }
    bool after_hip = false;
    if (a.stream_dirty) {                                     // HIP work the kernel may depend on
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        a.stream_dirty = false;
        a.stream_syncs++;
        after_hip = true;
    }
    const uint64_t idx = hsa_queue_add_write_index_relaxed(a.q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(a.q) >= a.q->size - 1) {}
    char *ka = a.karg + (idx & (a.q->size - 1)) * SLOT;
    memcpy(ka, buf, k.ksize);
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)a.q->base_address + (idx & (a.q->size - 1));
    p->workgroup_size_x = (uint16_t)block.x;
    p->workgroup_size_y = (uint16_t)block.y;
    p->workgroup_size_z = (uint16_t)block.z;
    p->grid_size_x = grid.x * block.x;
    p->grid_size_y = grid.y * block.y;
    p->grid_size_z = grid.z * block.z;
    p->private_segment_size = k.prv;
    p->group_segment_size = k.grp + (uint32_t)lds;
    p->kernel_object = k.kobj;
    p->kernarg_address = ka;
    p->completion_signal = hsa_signal_t{0};
    _mm_sfence();                                             // the write-combined kernarg stores land first
    // fences: kernel -> kernel on this device needs agent scope only (a system-scope acquire invalidates the L2 at
    // every kernel start); system scope to acquire what HIP's copies wrote, and at the drain (the host reads next)
    const uint16_t acq = after_hip ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                            (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = (uint16_t)((grid.z > 1 || block.z > 1 ? 3 : grid.y > 1 || block.y > 1 ? 2 : 1)
                                      << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(a.q->doorbell_signal, idx);
    a.submitted++;
    a.dispatches++;
    return true;
}

void aql_fallback_counted() { aql().fallbacks++; }

}  // namespace ghip
