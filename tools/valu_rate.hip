// valu_rate.hip — VALU issue rate per SIMD vs waves per SIMD (independent v_fma_f32 / v_cvt_f32_i32
// streams), and the same beside a stream of v_mfma_i32_32x32x32_i8 (one per 16 VALU).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && ./tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

typedef float f2 __attribute__((ext_vector_type(2)));
template <int MODE>  // 0: fma chain x8 independent, 1: cvt, 2: fma + mfma, 3: v_pk_fma_f32 (2 elements)
__global__ void k(float *out, int iters, long long *cyc) {
    float a[8];
    int ia[8];
    for (int i = 0; i < 8; i++) { a[i] = threadIdx.x * 0.001f + i; ia[i] = threadIdx.x + i; }
    const float m = 1.0001f, c = 0.5f;
    i32x16 acc = {};
    i32x4 op = {(int)threadIdx.x, 1, 2, 3};
    long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; it++) {
        if (MODE == 2) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(op, op, acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 2; r++) {
            if (MODE == 3) {
#pragma unroll
                for (int i = 0; i < 8; i += 2) {   // 4 packed instructions = 8 elements
                    f2 v = {a[i], a[i + 1]};
                    v = __builtin_elementwise_fma(v, f2{m, m}, f2{c, c});
                    v = __builtin_elementwise_fma(v, f2{m, m}, f2{c, c});
                    a[i] = v.x; a[i + 1] = v.y;
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (MODE == 1) a[i] += (float)(ia[i] + it);
                else a[i] = fmaf(a[i], m, c);
            }
        }
    }
    long long t1 = __builtin_readcyclecounter();
    float s = 0;
    for (int i = 0; i < 8; i++) s += a[i];
    if (MODE == 2) s += acc[0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *out; long long *cyc;
    CK(hipMalloc(&out, 1 << 24)); CK(hipMalloc(&cyc, 1 << 16));
    const int iters = 4096;
    for (int mode = 0; mode < 4; mode++) {
        for (int wps : {1, 2, 4}) {   // waves per SIMD: block = 4*wps waves on one CU
            const int threads = 256 * wps;
            hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            auto launch = [&]() {
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(threads), 0, 0, out, iters, cyc);
                else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(threads), 0, 0, out, iters, cyc);
                else if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(threads), 0, 0, out, iters, cyc);
                else hipLaunchKernelGGL(k<3>, dim3(256), dim3(threads), 0, 0, out, iters, cyc);
            };
            launch(); CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            long long c0; CK(hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost));
            // VALU instrs per wave: iters*16 (mode 1: cvt+add = 2 per element -> 32)
            // VALU instrs per wave: fma 16 per iter; cvt+add 32; pk: 8 packed (16 elements)
            const double vinst = (double)iters * (mode == 1 ? 32 : mode == 3 ? 8 : 16);
            printf("mode %d (%s) waves/SIMD %d: %.1f us, %lld cyc per wave -> %.2f cyc per VALU per wave, %.2f per SIMD\n",
                   mode, mode == 0 ? "fma" : mode == 1 ? "cvt+add" : mode == 2 ? "fma+mfma" : "pk_fma", wps, ms * 1e3, c0, c0 / vinst,
                   c0 / vinst / wps);
        }
    }
    return 0;
}
