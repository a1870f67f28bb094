// launch_floor.hip — cost of a dependent chain of kernels on one stream (eager and hipGraph),
// for several grid shapes.  hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/lf
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void empty_k(float *p) { if (p && threadIdx.x == 1234567) p[0] = 1.0f; }
__global__ void touch_k(float *p) { if (threadIdx.x == 0) p[blockIdx.x] += 1.0f; }
int main() {
    float *buf; CK(hipMalloc(&buf, 1 << 24));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int NK = 224;
    struct Cfg { int grid, block, lds; int touch; } cfgs[] = {
        {1, 64, 0, 0}, {256, 256, 0, 0}, {256, 1024, 0, 0}, {1024, 256, 0, 0}, {256, 1024, 5120, 0},
        {512, 1024, 0, 0}, {256, 256, 0, 1}, {2048, 256, 0, 0}};
    for (auto c : cfgs) {
        for (int graph = 0; graph < 2; graph++) {
            auto launch_all = [&]() {
                for (int i = 0; i < NK; i++) {
                    if (c.touch) hipLaunchKernelGGL(touch_k, dim3(c.grid), dim3(c.block), c.lds, s, buf);
                    else hipLaunchKernelGGL(empty_k, dim3(c.grid), dim3(c.block), c.lds, s, buf);
                }
            };
            hipGraphExec_t ge = nullptr; hipGraph_t g = nullptr;
            if (graph) {
                CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                launch_all();
                CK(hipStreamEndCapture(s, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            }
            for (int w = 0; w < 3; w++) { if (graph) CK(hipGraphLaunch(ge, s)); else launch_all(); }
            CK(hipStreamSynchronize(s));
            const int R = 20;
            CK(hipEventRecord(a, s));
            for (int r = 0; r < R; r++) { if (graph) CK(hipGraphLaunch(ge, s)); else launch_all(); }
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            printf("grid %5d block %4d lds %5d touch %d %s: %.3f us per kernel\n", c.grid, c.block, c.lds, c.touch,
                   graph ? "graph" : "eager", ms * 1e3 / (R * NK));
            if (graph) { hipGraphExecDestroy(ge); hipGraphDestroy(g); }
        }
    }
    return 0;
}
