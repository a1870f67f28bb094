// LDS-DMA streaming microbenchmark (the decode engine's loader, q4_0_engine.hip, in isolation): one workgroup per
// CU, each streaming its own contiguous slice of a 3.6 GB buffer into a 128 KiB LDS ring, nothing consuming.
//   hipcc -O3 --offload-arch=gfx950 tools/ldsdma_mb.hip -o tools/ldsdma_mb && tools/ldsdma_mb
// Variants: asm global_load_lds_dwordx4 with D lines (1 KiB) in flight, the buffer_load ... lds builtin, nt, 1 or 4
// loader waves per CU, and register loads (global_load_dwordx4, 16 waves) for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr unsigned RING = 128u * 1024u;

template <int NT>
__device__ __forceinline__ void dma(const void *g, unsigned lds) {
    unsigned keep;
    if (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

// W loader waves per workgroup, each streaming an interleaved 1/W of the CU's slice, D lines in flight per wave
// CTL: 1 = a ds_read_b128 + s_waitcnt lgkmcnt(0) of a control word per line (the engine loader's ring-space check),
// 2 = a ds_write_b32 per line (its landed publication), 3 = both
template <int D, int NT, int W, int BUF, int CTL = 0>
__global__ __launch_bounds__(64 * W) void k_stream(const char *src, size_t per_cu, unsigned *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const char *base = src + (size_t)blockIdx.x * per_cu;
    const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void_t *)lds);
    const unsigned nlines = (unsigned)(per_cu / 1024);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0, (int)per_cu, 0x00020000);
    unsigned issued = 0;
    for (unsigned i = w; i < nlines; i += W) {
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + ((i * 1024u) & (RING - 1)));
        if (BUF)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)((char *)lds + ((i * 1024u) & (RING - 1))), 16,
                                                     i * 1024u + lane * 16, 0, 0, NT ? 2 : 0);
        else
            dma<NT>(base + (size_t)i * 1024 + lane * 16, dst);
        if (++issued > (unsigned)D) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
        if (CTL & 1) {
            uint4 v;
            const unsigned a = lds0 + RING + 64;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
            if (v.x == 0x9999u) sink[0] = v.y;
        }
        if (CTL & 2) {
            const unsigned a = lds0 + RING + 128;
            asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(issued) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0 && lds[0] == 0x12345678u) sink[blockIdx.x] = 1;
}

// the engine's access pattern: the slice is read as 72 KiB units (32 rows of a K = 4096 q4_0 matrix), CU c taking
// units c, c + CUs, c + 2 CUs, ... of one big array (the round-robin deal of a matrix's units), one buffer
// descriptor per unit; CHK = control words read every 8 lines (as the engine loader does)
template <int D, int UNITKB>
__global__ __launch_bounds__(64) void k_units(const char *src, size_t per_cu, unsigned *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    const int lane = threadIdx.x & 63;
    const unsigned nunits = (unsigned)(per_cu / (UNITKB * 1024));
    unsigned issued = 0;
    for (unsigned u = 0; u < nunits; u++) {
        const char *ub = src + ((size_t)u * gridDim.x + blockIdx.x) * (UNITKB * 1024);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(ub), 0, UNITKB * 1024, 0x00020000);
        for (unsigned i = 0; i < (unsigned)UNITKB; i++) {
            const unsigned s0 = (u * UNITKB + i) * 1024u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t *)((char *)lds + (s0 & (RING - 1))), 16,
                                                     i * 1024u + lane * 16, 0, 0, 0);
            if (++issued > (unsigned)D && (issued & 7) == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0 && lds[0] == 0x12345678u) sink[blockIdx.x] = 1;
}

// reference: register streaming, 16 waves, 4 x 16 B per lane in flight
__global__ __launch_bounds__(1024) void k_regs(const char *src, size_t per_cu, unsigned *sink) {
    const char *base = src + (size_t)blockIdx.x * per_cu;
    const size_t n16 = per_cu / 16;
    unsigned acc = 0;
    for (size_t i = threadIdx.x; i < n16; i += 4 * 1024) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = i + k * 1024 < n16 ? reinterpret_cast<const uint4 *>(base)[i + k * 1024] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) acc ^= v[k].x ^ v[k].w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t per_cu = (size_t)14 * 1024 * 1024;   // 14 MiB per CU (the engine's LLaMA-7B stream)
    const size_t total = per_cu * cus;
    char *buf;
    unsigned *sink;
    CK(hipMalloc(&buf, total));
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipMemset(buf, 1, total));
    printf("CUs %d, %.2f GB streamed per run\n", cus, total / 1e9);
#define RUN(NAME, ...)                                                                                          \
    {                                                                                                           \
        auto kern = __VA_ARGS__;                                                                                \
        CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, RING + 256));    \
        const int W = NAME##_W;                                                                                 \
        float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * W), RING + 256, 0, buf, per_cu, sink); }, 5); \
        printf("%-40s %8.3f ms  %7.2f TB/s  %6.1f GB/s per CU\n", #NAME, ms, total / ms / 1e9, per_cu / ms / 1e6); \
    }
    constexpr int glds_d8_W = 1, glds_d16_W = 1, glds_d40_W = 1, glds_d60_W = 1, glds_d40_nt_W = 1, buf_d40_W = 1,
                  glds4_d16_W = 4, glds4_d40_W = 4, glds2_d40_W = 2, glds_d40_rd_W = 1, glds_d40_wr_W = 1,
                  glds_d40_rdwr_W = 1, buf_d40_rdwr_W = 1, units72_d40_W = 1, units72_d56_W = 1, units192_d40_W = 1,
                  units8_d40_W = 1;
    RUN(glds_d8, k_stream<8, 0, 1, 0>);
    RUN(glds_d16, k_stream<16, 0, 1, 0>);
    RUN(glds_d40, k_stream<40, 0, 1, 0>);
    RUN(glds_d60, k_stream<60, 0, 1, 0>);
    RUN(glds_d40_nt, k_stream<40, 1, 1, 0>);
    RUN(buf_d40, k_stream<40, 0, 1, 1>);
    RUN(glds2_d40, k_stream<40, 0, 2, 0>);
    RUN(glds4_d16, k_stream<16, 0, 4, 0>);
    RUN(glds4_d40, k_stream<40, 0, 4, 0>);
    RUN(glds_d40_rd, k_stream<40, 0, 1, 0, 1>);
    RUN(glds_d40_wr, k_stream<40, 0, 1, 0, 2>);
    RUN(glds_d40_rdwr, k_stream<40, 0, 1, 0, 3>);
    RUN(buf_d40_rdwr, k_stream<40, 0, 1, 1, 3>);
    RUN(units72_d40, k_units<40, 72>);
    RUN(units72_d56, k_units<56, 72>);
    RUN(units192_d40, k_units<40, 192>);
    RUN(units8_d40, k_units<40, 8>);
    {
        float ms = timeit([&] { hipLaunchKernelGGL(k_regs, dim3(cus), dim3(1024), 0, 0, buf, per_cu, sink); }, 5);
        printf("%-40s %8.3f ms  %7.2f TB/s  %6.1f GB/s per CU\n", "regs16waves", ms, total / ms / 1e9, per_cu / ms / 1e6);
    }
    return 0;
}
