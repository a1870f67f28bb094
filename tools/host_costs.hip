// host_costs.hip — host-side cost of the HIP calls on the tensor-ABI hot path (one per ggml node
// at full offload): hipSetDevice, hipGetDevice, hipGetLastError, an empty kernel launch.
//   hipcc --offload-arch=gfx950 -O2 tools/host_costs.hip -o tools/host_costs && tools/host_costs
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <mutex>
__global__ void k_empty(float *p) { if (p && threadIdx.x == 1024) p[0] = 1.0f; }
template <class F> double per_call_us(int n, F f) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}
int main() {
    hipStream_t s;
    hipSetDevice(0);
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
    hipStreamSynchronize(s);
    std::mutex mu;
    int d = 0;
    printf("hipSetDevice(same)   %.3f us\n", per_call_us(100000, [&] { (void)hipSetDevice(0); }));
    printf("hipGetDevice         %.3f us\n", per_call_us(100000, [&] { (void)hipGetDevice(&d); }));
    printf("hipGetLastError      %.3f us\n", per_call_us(100000, [&] { (void)hipGetLastError(); }));
    printf("mutex lock+unlock    %.3f us\n", per_call_us(100000, [&] { std::lock_guard<std::mutex> l(mu); }));
    for (int grid : {1, 64, 1024}) {
        double us = per_call_us(20000, [&] { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, nullptr); });
        hipStreamSynchronize(s);
        printf("launch grid %5d    %.3f us (host, back to back)\n", grid, us);
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 20000; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, nullptr);
    hipStreamSynchronize(s);
    printf("20000 launches incl. drain: %.3f us each (device-bound if > host)\n",
           std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 20000);
    return 0;
}
