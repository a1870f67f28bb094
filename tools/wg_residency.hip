// wg_residency.hip — how many waves / workgroups are resident per CU at once?  Every wave records its
// start and end (s_memrealtime, 100 MHz) and where it ran (HW_ID, XCC_ID) while spinning for 3 us;
// the peak count of overlapping waves per CU is the residency.
//   hipcc --offload-arch=gfx950 -O3 tools/wg_residency.hip -o tools/wg_residency && ./tools/wg_residency
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ const uint4 *g_src;   // streamed by MODE 2 (set by the host)
template <int REGS>
__global__ void k_spin(unsigned long long *out, int spin) {
    extern __shared__ float lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (REGS == 1 || REGS >= 3) asm volatile("" ::: "v42", "s69");   // the q|k|v GEMV's 43 VGPRs / 70 SGPRs
    if constexpr (REGS == 2) asm volatile("" ::: "v63", "s95");
    if constexpr (REGS == 3) __syncthreads();                                     // a workgroup barrier
    if constexpr (REGS == 4) {                                                    // stream 36 KB per wave
        uint4 acc = {0, 0, 0, 0};
        const uint4 *p = g_src + ((size_t)(blockIdx.x * blockDim.x + threadIdx.x) * 36);
#pragma unroll 4
        for (int i = 0; i < 36; i++) {
            const uint4 v = p[i];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        if (acc.x == 0x12345u) lds[0] = 1.0f;
    }
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(1);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);    // HW_REG_XCC_ID
        volatile unsigned long long *o = out + 4 * w;
        o[0] = t0;
        o[1] = t1;
        o[2] = hw;
        o[3] = xcc;
        if (blockDim.x > 64) lds[threadIdx.x & 63] = 0.0f;
    }
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("%s: %d CUs, maxThreadsPerMultiProcessor %d, regsPerMultiprocessor %d, sharedMemPerMultiprocessor %zu\n",
           p.gcnArchName, p.multiProcessorCount, p.maxThreadsPerMultiProcessor, p.regsPerMultiprocessor,
           p.sharedMemPerMultiprocessor);
    unsigned long long *d;
    CK(hipMalloc(&d, 1 << 26));
    struct Cfg { int wgs, threads, lds, regs, pred; };
    const Cfg cfgs[] = {{512, 1024, 5120, 1, 1}, {512, 1024, 5120, 3, 1}, {512, 1024, 5120, 4, 1},
                        {256, 1024, 5120, 4, 1}, {1024, 512, 5120, 4, 1}};
    void (*kern[5])(unsigned long long *, int) = {k_spin<0>, k_spin<1>, k_spin<2>, k_spin<3>, k_spin<4>};
    uint4 *src;
    CK(hipMalloc(&src, (size_t)8192 * 64 * 36 * 16));            // 302 MB: every wave its own 36 KB
    CK(hipMemset(src, 1, (size_t)8192 * 64 * 36 * 16));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_src), &src, sizeof(src)));
    for (const Cfg &c : cfgs) {
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern[c.regs], c.threads, c.lds));
        for (int rep = 0; rep < 3; rep++) {
            CK(hipMemset(d, 0, 1 << 26));
            // c.pred: the launch follows another one on the same stream (as in the bench's chain)
            if (c.pred) hipLaunchKernelGGL(kern[c.regs], dim3(256), dim3(1024), c.lds, 0, d + (1 << 22), 300);
            hipLaunchKernelGGL(kern[c.regs], dim3(c.wgs), dim3(c.threads), c.lds, 0, d, 300);
            CK(hipDeviceSynchronize());
        }
        const int waves = c.wgs * c.threads / 64;
        std::vector<unsigned long long> h(4 * (size_t)waves);
        CK(hipMemcpy(h.data(), d, 32ull * waves, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int w = 0; w < waves; w++) t0 = std::min(t0, h[4 * w]);
        // per CU (xcc, se, sh, cu): events (+1 at start, -1 at end) -> peak concurrency
        std::map<unsigned, std::vector<std::pair<unsigned long long, int>>> ev;
        int late = 0;
        for (int w = 0; w < waves; w++) {
            const unsigned hw = (unsigned)h[4 * w + 2], xcc = (unsigned)h[4 * w + 3] & 0xF;
            const unsigned cu = (xcc << 16) | (hw & 0xFF00);             // cu_id [11:8], sh [12], se [15:13]
            ev[cu].push_back({h[4 * w], +1});
            ev[cu].push_back({h[4 * w + 1], -1});
            if (h[4 * w] - t0 > 200) late++;                              // started > 2 us after the first
        }
        int peak_min = 1 << 30, peak_max = 0;
        for (auto &kv : ev) {
            auto &v = kv.second;
            std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
            int cur = 0, pk = 0;
            for (auto &e : v) pk = std::max(pk, cur += e.second);
            peak_min = std::min(peak_min, pk);
            peak_max = std::max(peak_max, pk);
        }
        printf("pred %d regs %d wgs %5d x %4d threads (occupancy query %d WG/CU): %zu CUs used, peak resident waves per CU %d..%d, "
               "%d of %d waves started > 2 us late\n",
               c.pred, c.regs, c.wgs, c.threads, occ, ev.size(), peak_min, peak_max, late, waves);
    }
    return 0;
}
