// Host cost per kernel launch through three HIP entry points (round 5, e2e decode host walk): hipLaunchKernelGGL
// (what ghip::launch_k uses), hipModuleLaunchKernel on the function handle from hipGetFuncBySymbol with the
// arguments as one packed buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER), and hipExtLaunchKernel.  An empty kernel with
// a GEMV-like argument list; 20,000 launches per API in batches of 200 (a stream synchronize between batches,
// not timed), host wall time per launch.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

struct Args {
    const float *x; const unsigned char *w0, *w1, *w2; int a, b, c, d, e, f; float *y; long ldy;
};

__global__ void k_empty(const float *x, const unsigned char *w0, const unsigned char *w1, const unsigned char *w2, int a,
                        int b, int c, int d, int e, int f, float *y, long ldy) {
    if (a == -12345 && threadIdx.x == 0) y[ldy] = x[0] + (float)(w0[0] + w1[0] + w2[0] + b + c + d + e + f);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *y;
    CK(hipMalloc(&y, 4096));
    hipFunction_t f;
    CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void *>(k_empty)));
    const int batches = 100, per = 200;
    for (int round = 0; round < 3; round++) {
        for (int api = 0; api < 3; api++) {
            double ns = 0;
            for (int bt = 0; bt < batches; bt++) {
                CK(hipStreamSynchronize(s));
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < per; i++) {
                    if (api == 0) {
                        hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s, (const float *)y, (const unsigned char *)y,
                                           (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L);
                    } else if (api == 1) {
                        Args a{y, (const unsigned char *)y, (const unsigned char *)y, (const unsigned char *)y, i, 2, 3, 4, 5, 6, y, 7L};
                        size_t sz = sizeof(a);
                        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
                        (void)hipModuleLaunchKernel(f, 256, 1, 1, 1024, 1, 1, 0, s, nullptr, cfg);
                    } else {
                        const float *xp = y; const unsigned char *wp = (const unsigned char *)y; int ii = i, two = 2, three = 3,
                            four = 4, five = 5, six = 6; float *yp = y; long l = 7;
                        void *args[] = {&xp, &wp, &wp, &wp, &ii, &two, &three, &four, &five, &six, &yp, &l};
                        (void)hipExtLaunchKernel(reinterpret_cast<const void *>(k_empty), dim3(256), dim3(1024), args, 0, s,
                                                 nullptr, nullptr, 0);
                    }
                }
                ns += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
            }
            CK(hipStreamSynchronize(s));
            CK(hipGetLastError());
            const char *nm[] = {"hipLaunchKernelGGL", "hipModuleLaunchKernel(buffer)", "hipExtLaunchKernel"};
            printf("round %d %-30s %.3f us per launch\n", round, nm[api], ns / (batches * per) / 1e3);
        }
    }
    return 0;
}
