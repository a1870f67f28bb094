// Host cost of a raw AQL kernel dispatch (verdict r5 item 3: "measure a raw HSA AQL dispatch from the host before
// building a hook-path submission on it"), beside hipLaunchKernelGGL on the same empty kernel:
//   * the kernel object from a code object loaded through HSA (tools/aql_kernel.hip as a bare ELF, --no-gpu-bundle-output),
//   * an own HSA queue (hsa_queue_create, single producer), kernarg ring in the kernarg memory pool,
//   * per dispatch: reserve the write index, fill the packet + kernargs, publish the header with a release store,
//     ring the doorbell.
// 20,000 dispatches per path in batches of 200 (waits between batches untimed), host wall time per dispatch.
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c -O2 tools/aql_kernel.hip -o tools/aql_kernel.hsaco
//   hipcc -O2 --offload-arch=gfx950 tools/aql_dispatch_cost.hip -o tools/aql_dispatch_cost -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CKH(x) do { hsa_status_t e_ = (x); if (e_ != HSA_STATUS_SUCCESS) { const char *m = nullptr; hsa_status_string(e_, &m); \
    printf("HSA error %s at %d: %s\n", m ? m : "?", __LINE__, #x); return 1; } } while (0)
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Args {     // the GEMV-like 12-argument list of tools/launch_api_cost.hip
    const float *x; const unsigned char *w0, *w1, *w2; int a, b, c, d, e, f; float *y; long ldy;
};

extern "C" __global__ void k_empty_hip(const float *x, const unsigned char *w0, const unsigned char *w1,
                                       const unsigned char *w2, int a, int b, int c, int d, int e, int f, float *y, long ldy) {
    if (a == -12345 && threadIdx.x == 0) y[ldy] = x[0] + (float)(w0[0] + w1[0] + w2[0] + b + c + d + e + f);
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_amd_memory_pool_t g_kernarg_pool{};
static bool g_have_pool = false;

static hsa_status_t find_agents(hsa_agent_t agent, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = agent;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = agent;
    return HSA_STATUS_SUCCESS;
}
static hsa_amd_memory_pool_t g_dev_pool{};
static bool g_have_dev_pool = false;
static hsa_status_t find_dev_pool(hsa_amd_memory_pool_t pool, void *) {    // the GPU's coarse-grained VRAM pool
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g_have_dev_pool) {
        g_dev_pool = pool;
        g_have_dev_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t pool, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_pool) {
        g_kernarg_pool = pool;
        g_have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}

int main(int argc, char **argv) {
    const char *co_path = argc > 1 ? argv[1] : "tools/aql_kernel.hsaco";
    // HIP first (it initialises the runtime the HSA calls share)
    float *y;
    CK(hipMalloc(&y, 4096));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CKH(hsa_init());
    CKH(hsa_iterate_agents(find_agents, nullptr));
    CKH(hsa_amd_agent_iterate_memory_pools(g_cpu, find_kernarg_pool, nullptr));
    if (!g_have_pool) { printf("no kernarg pool\n"); return 1; }
    // the kernel object from the code object
    FILE *f = fopen(co_path, "rb");
    if (!f) { printf("cannot open %s\n", co_path); return 1; }
    std::vector<char> co;
    {
        char buf[65536];
        size_t n;
        while ((n = fread(buf, 1, sizeof buf, f)) > 0) co.insert(co.end(), buf, buf + n);
        fclose(f);
    }
    hsa_code_object_reader_t reader;
    CKH(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader));
    hsa_executable_t exe;
    CKH(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    CKH(hsa_executable_load_agent_code_object(exe, g_gpu, reader, nullptr, nullptr));
    CKH(hsa_executable_freeze(exe, nullptr));
    hsa_executable_symbol_t sym;
    CKH(hsa_executable_get_symbol_by_name(exe, "k_empty_aql.kd", &g_gpu, &sym));
    uint64_t kobj = 0;
    uint32_t ka_size = 0, grp = 0, prv = 0;
    CKH(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
    CKH(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &ka_size));
    CKH(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &grp));
    CKH(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &prv));
    // own queue + kernarg ring
    hsa_queue_t *q;
    CKH(hsa_queue_create(g_gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    const uint32_t qmask = q->size - 1;
    const size_t slot = ka_size <= 256 ? 256 : ((size_t)ka_size + 255) & ~(size_t)255;   // hidden args included
    char *karg = nullptr;
    CKH(hsa_amd_memory_pool_allocate(g_kernarg_pool, slot * q->size, 0, (void **)&karg));
    CKH(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, karg));
    // kernargs in VRAM (what HIP does by default on this GPU family) for the device-side comparison, written by the
    // CPU through the large-BAR mapping; skipped where the pool or the CPU access is not available
    char *karg_dev = nullptr;
    if (hsa_amd_agent_iterate_memory_pools(g_gpu, find_dev_pool, nullptr) == HSA_STATUS_SUCCESS && g_have_dev_pool &&
        hsa_amd_memory_pool_allocate(g_dev_pool, slot * q->size, 0, (void **)&karg_dev) == HSA_STATUS_SUCCESS) {
        if (hsa_amd_agents_allow_access(1, &g_cpu, nullptr, karg_dev) != HSA_STATUS_SUCCESS) {
            hsa_amd_memory_pool_free(karg_dev);
            karg_dev = nullptr;
        }
    }
    printf("VRAM kernargs: %s\n", karg_dev ? "yes" : "no");
    hsa_signal_t done;
    CKH(hsa_signal_create(1, 0, nullptr, &done));
    printf("kernel object %#llx, kernarg %u B, group %u, private %u, queue size %u\n", (unsigned long long)kobj, ka_size,
           grp, prv, q->size);

    auto aql = [&](int i, bool last) {
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
        hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & qmask);
        Args a{y, (const unsigned char *)y, (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L};
        char *ka = karg + (idx & qmask) * slot;
        memset(ka, 0, slot);                       // hidden arguments zero (the kernel reads none)
        memcpy(ka, &a, sizeof a);
        p->workgroup_size_x = 1024;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = 256 * 1024;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->private_segment_size = prv;
        p->group_segment_size = grp;
        p->kernel_object = kobj;
        p->kernarg_address = ka;
        p->completion_signal = last ? done : hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (1 << HSA_PACKET_HEADER_BARRIER) |
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
    };
    const int batches = 100, per = 200;
    for (int round = 0; round < 3; round++) {
        for (int api = 0; api < 2; api++) {
            double ns = 0;
            for (int bt = 0; bt < batches; bt++) {
                CK(hipStreamSynchronize(s));
                hsa_signal_store_relaxed(done, 1);
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < per; i++) {
                    if (api == 0)
                        hipLaunchKernelGGL(k_empty_hip, dim3(256), dim3(1024), 0, s, (const float *)y, (const unsigned char *)y,
                                           (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L);
                    else
                        aql(i, i == per - 1);
                }
                auto t1 = std::chrono::steady_clock::now();
                ns += std::chrono::duration<double, std::nano>(t1 - t0).count();
                if (api == 1)      // bounded wait for the batch's last packet (5 s)
                    if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 5000000000ull, HSA_WAIT_STATE_ACTIVE) != 0) {
                        printf("AQL batch did not complete\n");
                        return 1;
                    }
            }
            printf("round %d %-28s %.3f us per dispatch (host)\n", round, api == 0 ? "hipLaunchKernelGGL" : "raw AQL (own queue)",
                   ns / (batches * per) / 1e3);
        }
    }
    // Device side: the time per DEPENDENT dispatch (barrier bit) of the same empty 256 x 1024 grid, back to back:
    // HIP (hipLaunchKernelGGL, events around 2,000 launches) against 2,000 AQL packets written first and released by
    // one doorbell, with system-scope and with agent-scope acquire/release fences (what the CP does at every kernel
    // boundary: HIP's packets carry system scope), and without the barrier bit (no ordering, for reference).
    {
        const int n = 2000;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int round = 0; round < 3; round++) {
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < n; i++)
                hipLaunchKernelGGL(k_empty_hip, dim3(256), dim3(1024), 0, s, (const float *)y, (const unsigned char *)y,
                                   (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("round %d device, hipLaunchKernelGGL back to back   %.3f us per kernel\n", round, ms * 1e3f / n);
            const char *names[4] = {"AQL, barrier, system-scope fences", "AQL, barrier, agent-scope fences ",
                                    "AQL, no barrier, agent-scope      ", "AQL, barrier, system, VRAM kernargs"};
            for (int mode = 0; mode < (karg_dev ? 4 : 3); mode++) {
                char *kbase = mode == 3 ? karg_dev : karg;
                const uint16_t scope = (mode == 0 || mode == 3) ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT;
                const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                        ((mode != 2 ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                                        (scope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                        (scope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
                // the last packet: barrier + system scope so the signal sees everything
                const uint16_t last_header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                             (1 << HSA_PACKET_HEADER_BARRIER) |
                                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
                const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
                hsa_signal_store_relaxed(done, 1);
                uint64_t first = 0, idx = 0;
                for (int i = 0; i < n; i++) {
                    idx = hsa_queue_add_write_index_relaxed(q, 1);
                    if (i == 0) first = idx;
                    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
                    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & qmask);
                    Args a{y, (const unsigned char *)y, (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L};
                    char *ka = kbase + (idx & qmask) * slot;
                    memcpy(ka, &a, sizeof a);                    // (the kernel reads no hidden argument)
                    p->workgroup_size_x = 1024; p->workgroup_size_y = 1; p->workgroup_size_z = 1;
                    p->grid_size_x = 256 * 1024; p->grid_size_y = 1; p->grid_size_z = 1;
                    p->private_segment_size = prv;
                    p->group_segment_size = grp;
                    p->kernel_object = kobj;
                    p->kernarg_address = ka;
                    p->completion_signal = i == n - 1 ? done : hsa_signal_t{0};
                    __atomic_store_n((uint32_t *)p, (uint32_t)(i == n - 1 ? last_header : header) | ((uint32_t)setup << 16),
                                     __ATOMIC_RELEASE);
                }
                (void)first;
                const auto t0 = std::chrono::steady_clock::now();
                hsa_signal_store_screlease(q->doorbell_signal, idx);            // one doorbell for all
                if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 5000000000ull, HSA_WAIT_STATE_ACTIVE) != 0) {
                    printf("AQL batch did not complete\n");
                    return 1;
                }
                const auto t1 = std::chrono::steady_clock::now();
                printf("round %d device, %s %.3f us per kernel\n", round, names[mode],
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
            }
        }
    }
    CK(hipStreamSynchronize(s));
    hsa_signal_destroy(done);
    hsa_queue_destroy(q);
    hsa_amd_memory_pool_free(karg);
    hsa_executable_destroy(exe);
    hsa_code_object_reader_destroy(reader);
    return 0;
}
