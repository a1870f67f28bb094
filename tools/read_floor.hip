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

int main() {
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    unsigned *out; CK(hipMalloc(&out, 64));
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
            {2, g16, 1024, 0}, {3, g16, 1024, 0}, {4, g16, 1024, 0}, {4, g16, 1024, 20480}};
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
