// read_floor.hip — HBM streaming floor of one launch in a dependent graph chain, at the decode
// GEMV byte counts: how long does a kernel that only reads S bytes (and writes one dword per
// wave) take, per launch, for several access shapes?  No activation, no math.
//   hipcc --offload-arch=gfx950 -O3 tools/read_floor.hip -o /tmp/rf && /tmp/rf
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// shape 0: coalesced, thread t reads 16 B at 16*(t + k*T) with U loads in flight
template <int U>
__global__ __launch_bounds__(1024) void rd_coalesced(const u32x4 *__restrict__ p, size_t n16, unsigned *out) {
    const size_t T = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (; i + (U - 1) * T < n16; i += U * T) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(p + i + u * T);
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n16; i += T) { u32x4 v = p[i]; acc ^= v.x + v.y + v.z + v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

// shape 1: the GEMV pattern: one wave per row (rowbytes), lane l reads the 36-byte pair l of each
// 64-pair chunk (b128, b128, b32), rows strided by the number of waves in the grid
__global__ __launch_bounds__(1024) void rd_rows(const unsigned char *__restrict__ p, int M, int rowbytes, unsigned *out) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int nw = gridDim.x * (blockDim.x >> 6);
    unsigned acc = 0;
    const int npairs = rowbytes / 36;
    for (int r = wave; r < M; r += nw) {
        const unsigned char *row = p + (size_t)r * rowbytes;
        for (int q = lane; q < npairs; q += 64) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(row + 36 * q);
            const u32x4 b = *reinterpret_cast<const u32x4 *>(row + 36 * q + 16);
            const unsigned c = *reinterpret_cast<const unsigned *>(row + 36 * q + 32);
            acc ^= a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// shape 2..: rd_rows plus one feature of the GEMV each (bisecting the GEMV's excess over the floor)
//  F_BUF: buffer loads through a per-row descriptor; F_RED: per-row wave sum (DPP via __shfl_xor) + lane-0
//  store of one float per row to y
template <bool F_BUF, bool F_RED>
__global__ __launch_bounds__(1024) void rd_rows_f(const unsigned char *__restrict__ p, int M, int rowbytes, float *y) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int nw = gridDim.x * (blockDim.x >> 6);
    const int npairs = rowbytes / 36;
    unsigned accx = 0;
    for (int r = wave; r < M; r += nw) {
        const unsigned char *row = p + (size_t)r * rowbytes;
        unsigned acc = 0;
        for (int q = lane; q < npairs + 63 - 63 * 0 && q - lane < npairs; q += 64) {
            u32x4 a, b; unsigned c;
            if (F_BUF) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)row, 0, rowbytes, 0x00020000);
                a = __builtin_amdgcn_raw_buffer_load_b128(rs, 36 * q, 0, 0);
                b = __builtin_amdgcn_raw_buffer_load_b128(rs, 36 * q + 16, 0, 0);
                c = __builtin_amdgcn_raw_buffer_load_b32(rs, 36 * q + 32, 0, 0);
            } else {
                if (q >= npairs) break;
                a = *reinterpret_cast<const u32x4 *>(row + 36 * q);
                b = *reinterpret_cast<const u32x4 *>(row + 36 * q + 16);
                c = *reinterpret_cast<const unsigned *>(row + 36 * q + 32);
            }
            acc ^= a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c;
        }
        if (F_RED) {
            float f = (float)acc;
            for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o);
            if (lane == 0) y[r] = f;
        } else {
            accx ^= acc;
        }
    }
    if (!F_RED && accx == 0x12345678u) y[0] = 1.0f;
}

// shape 5/6: the workgroup's contiguous row range [b*M/grid, (b+1)*M/grid) read as aligned 16-B pieces
// (thread t: piece t + k*blockDim), U pieces in flight; 5 = into registers, 6 = LDS-DMA into a 1-KiB
// slot per wave (global_load_lds_dwordx4, no VGPR destination)
typedef __attribute__((address_space(3))) void lds_void_t;
template <int U, bool DMA>
__global__ __launch_bounds__(1024) void rd_slab(const unsigned char *__restrict__ p, int M, int rowbytes, unsigned *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    const size_t b0 = ((size_t)blockIdx.x * M / gridDim.x) * rowbytes & ~(size_t)15;
    const size_t b1 = ((size_t)(blockIdx.x + 1) * M / gridDim.x) * rowbytes;
    const int n16 = (int)((b1 - b0 + 15) / 16);
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p + b0);
    const int T = blockDim.x;
    unsigned acc = 0;
    int i = threadIdx.x;
    if (DMA) {
        const int wave = threadIdx.x >> 6;
        for (; i - (int)(threadIdx.x & 63) < n16; i += T) {
            const int ii = i < n16 ? i : n16 - 1;
            __builtin_amdgcn_global_load_lds((const void *)(q + ii), (lds_void_t *)(sm + wave * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc = sm[threadIdx.x * 4];
    } else {
        for (; i + (U - 1) * T < n16; i += U * T) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = q[i + u * T];
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        }
        for (; i < n16; i += T) { u32x4 v = q[i]; acc ^= v.x + v.y + v.z + v.w; }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// shape 7: grid-stride over the matrix's 36-byte block pairs (thread t: pairs t + k*T; b128, b128, b32);
// shape 8: shape 0 with default-policy loads (no nt)
template <bool NTL>
__global__ __launch_bounds__(1024) void rd_pairs(const unsigned char *__restrict__ p, size_t npairs_total, unsigned *out) {
    const size_t T = (size_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs_total; i += T) {
        const unsigned char *q = p + 36 * i;
        u32x4 a, b; unsigned c;
        if (NTL) {
            a = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(q));
            b = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(q + 16));
            c = __builtin_nontemporal_load(reinterpret_cast<const unsigned *>(q + 32));
        } else {
            a = *reinterpret_cast<const u32x4 *>(q);
            b = *reinterpret_cast<const u32x4 *>(q + 16);
            c = *reinterpret_cast<const unsigned *>(q + 32);
        }
        acc ^= a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(1024) void rd_coalesced_plain(const u32x4 *__restrict__ p, size_t n16, unsigned *out) {
    const size_t T = (size_t)gridDim.x * blockDim.x;
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += T) {
        u32x4 v = p[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// shape 10: per-wave private LDS ring of SLOTS x SKB KiB, filled by LDS-DMA (global_load_lds_dwordx4, nt
// when NTL) with 16-B aligned pieces of the workgroup's contiguous row range, consumed by ds_read_b32 of
// every dword (a stand-in for the pair reads), refilled behind a counted vmcnt; no VGPR weight traffic
template <int WAVES, int SLOTS, int SKB, bool NTL>
__global__ __launch_bounds__(WAVES * 64) void rd_dma_ring(const unsigned char *__restrict__ p, int M, int rowbytes,
                                                         unsigned *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t b0 = ((size_t)blockIdx.x * M / gridDim.x) * rowbytes & ~(size_t)15;
    const size_t b1 = ((size_t)(blockIdx.x + 1) * M / gridDim.x) * rowbytes;
    constexpr int IB = SKB * 1024;                                   // bytes per item (one slot)
    const int nitems = (int)((b1 - b0 + IB - 1) / IB);
    unsigned char *ring = sm + wave * SLOTS * IB;
    const int last16 = (int)((b1 - b0 + 15) / 16) - 1;
    auto issue = [&](int it, int slot) {
        const int item = it * WAVES + wave;
#pragma unroll
        for (int j = 0; j < SKB; j++) {
            int piece = item * (IB / 16) + j * 64 + lane;
            piece = piece < last16 ? piece : last16;
            __builtin_amdgcn_global_load_lds((const void *)(p + b0 + 16 * (size_t)piece),
                                             (lds_void_t *)(ring + slot * IB + j * 1024), 16, 0, NTL ? 2 : 0);
        }
    };
    const int myitems = nitems > wave ? (nitems - 1 - wave) / WAVES + 1 : 0;
    unsigned acc = 0;
#pragma unroll
    for (int s = 0; s < SLOTS; s++) issue(s, s);                   // past-the-end items clamp (no traffic)
    for (int it = 0; it < myitems; it++) {
        const int slot = it % SLOTS;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((SLOTS - 1) * SKB) : "memory");
        const unsigned *d = reinterpret_cast<const unsigned *>(ring + slot * IB);
#pragma unroll
        for (int o = 0; o < IB / 256; o++) acc ^= d[o * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(it + SLOTS, slot);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    unsigned *out; CK(hipMalloc(&out, 64));
    CK(hipFuncSetAttribute((const void *)rd_dma_ring<8, 4, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    CK(hipFuncSetAttribute((const void *)rd_dma_ring<16, 4, 2, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    CK(hipFuncSetAttribute((const void *)rd_dma_ring<8, 4, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    float *yb; CK(hipMalloc(&yb, 1 << 20));
    struct Sz { const char *name; int M, K; } sizes[] = {
        {"wq|wk|wv 4096x12288", 12288, 4096}, {"wo 4096x4096", 4096, 4096},
        {"w1|w3 4096x22016", 22016, 4096}, {"w2 11008x4096", 4096, 11008}};
    const int NB = 32;  // distinct buffers per chain (> MALL)
    for (auto sz : sizes) {
        const int rowbytes = sz.K / 32 * 18;
        const size_t bytes = (size_t)sz.M * rowbytes;
        std::vector<unsigned char *> bufs(NB);
        for (auto &p : bufs) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 1, bytes)); }
        const int g16 = (sz.M + 15) / 16 < ncu * 2 ? (sz.M + 15) / 16 : ncu * 2;
        struct Cfg { int shape, grid, block, lds; } cfgs[] = {
            {0, ncu * 8, 256, 0}, {1, g16, 1024, 0}, {1, g16, 1024, 20480},
            {3, g16, 1024, 0},
            {7, ncu * 4, 256, 0},
            {8, ncu * 8, 256, 0}, {10, ncu, 8 * 64, 0}, {11, ncu, 16 * 64, 0}, {12, ncu * 2, 8 * 64, 0},
            {13, ncu, 8 * 64, 0}, {14, ncu * 2, 4 * 64, 0}};
        for (auto c : cfgs) {
            for (int U : {1, 2, 4}) {
                if (c.shape >= 1 && U != 1) continue;
                auto launch_all = [&]() {
                    for (int i = 0; i < NB; i++) {
                        if (c.shape == 1)
                            hipLaunchKernelGGL(rd_rows, dim3(c.grid), dim3(c.block), c.lds, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 2)
                            hipLaunchKernelGGL((rd_rows_f<true, false>), dim3(c.grid), dim3(c.block), c.lds, s, bufs[i], sz.M, rowbytes, yb);
                        else if (c.shape == 3)
                            hipLaunchKernelGGL((rd_rows_f<false, true>), dim3(c.grid), dim3(c.block), c.lds, s, bufs[i], sz.M, rowbytes, yb);
                        else if (c.shape == 4)
                            hipLaunchKernelGGL((rd_rows_f<true, true>), dim3(c.grid), dim3(c.block), c.lds, s, bufs[i], sz.M, rowbytes, yb);
                        else if (c.shape == 5 && U == 1)
                            hipLaunchKernelGGL((rd_slab<1, false>), dim3(c.grid), dim3(c.block), 0, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 5 && U == 2)
                            hipLaunchKernelGGL((rd_slab<2, false>), dim3(c.grid), dim3(c.block), 0, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 5)
                            hipLaunchKernelGGL((rd_slab<4, false>), dim3(c.grid), dim3(c.block), 0, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 7)
                            hipLaunchKernelGGL((rd_pairs<false>), dim3(c.grid), dim3(c.block), 0, s, bufs[i], bytes / 36, out);
                        else if (c.shape == 9)
                            hipLaunchKernelGGL((rd_pairs<true>), dim3(c.grid), dim3(c.block), 0, s, bufs[i], bytes / 36, out);
                        else if (c.shape == 8)
                            hipLaunchKernelGGL(rd_coalesced_plain, dim3(c.grid), dim3(c.block), 0, s, (const u32x4 *)bufs[i], bytes / 16, out);
                        else if (c.shape == 10)   // 8 waves x 4 slots x 4 KiB = 128 KiB, nt
                            hipLaunchKernelGGL((rd_dma_ring<8, 4, 4, true>), dim3(c.grid), dim3(c.block), 131072, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 11)   // 16 waves x 4 slots x 2 KiB, nt
                            hipLaunchKernelGGL((rd_dma_ring<16, 4, 2, true>), dim3(c.grid), dim3(c.block), 131072, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 12)   // 2 WG/CU: 8 waves x 2 slots x 4 KiB = 64 KiB, nt
                            hipLaunchKernelGGL((rd_dma_ring<8, 2, 4, true>), dim3(c.grid), dim3(c.block), 65536, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 13)   // as 10, default policy
                            hipLaunchKernelGGL((rd_dma_ring<8, 4, 4, false>), dim3(c.grid), dim3(c.block), 131072, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 14)   // 2 WG/CU: 4 waves x 4 slots x 4 KiB = 64 KiB, nt
                            hipLaunchKernelGGL((rd_dma_ring<4, 4, 4, true>), dim3(c.grid), dim3(c.block), 65536, s, bufs[i], sz.M, rowbytes, out);
                        else if (c.shape == 6)
                            hipLaunchKernelGGL((rd_slab<1, true>), dim3(c.grid), dim3(c.block), c.lds, s, bufs[i], sz.M, rowbytes, out);
                        else if (U == 1)
                            hipLaunchKernelGGL(rd_coalesced<1>, dim3(c.grid), dim3(c.block), 0, s, (const u32x4 *)bufs[i], bytes / 16, out);
                        else if (U == 2)
                            hipLaunchKernelGGL(rd_coalesced<2>, dim3(c.grid), dim3(c.block), 0, s, (const u32x4 *)bufs[i], bytes / 16, out);
                        else
                            hipLaunchKernelGGL(rd_coalesced<4>, dim3(c.grid), dim3(c.block), 0, s, (const u32x4 *)bufs[i], bytes / 16, out);
                    }
                };
                hipGraph_t g; hipGraphExec_t ge;
                CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                launch_all();
                CK(hipStreamEndCapture(s, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGetLastError());
                for (int w = 0; w < 3; w++) CK(hipGraphLaunch(ge, s));
                CK(hipStreamSynchronize(s));
                const int R = 20;
                CK(hipEventRecord(a, s));
                for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, s));
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms; CK(hipEventElapsedTime(&ms, a, b));
                const double us = ms * 1e3 / (R * NB);
                printf("%-22s shape %d grid %5d block %4d lds %5d U %d: %7.3f us/launch  %7.1f GB/s\n", sz.name, c.shape,
                       c.grid, c.block, c.lds, U, us, bytes / us / 1e3);
                CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
            }
        }
        for (auto p : bufs) CK(hipFree(p));
    }
    return 0;
}
