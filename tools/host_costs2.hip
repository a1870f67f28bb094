// host_costs2.hip — host cost per kernel launch when the queue is NOT full (bursts of 300 launches,
// the size of one full-offload decode eval, then a drain), by launch API, and the host cost of
// replaying the same 300 kernels as a HIP graph (incl. kernel-node parameter updates).
//   hipcc --offload-arch=gfx950 -O2 tools/host_costs2.hip -o tools/host_costs2 && tools/host_costs2
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <vector>
__global__ void k_small(float *p, int a, int b, long c) {
    if (p && threadIdx.x + blockIdx.x * 256 == 1u << 30) p[0] = (float)(a + b + c);
}
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
    hipStream_t s;
    hipSetDevice(0);
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    float *p = nullptr;
    hipMalloc(&p, 4096);
    const int B = 300, R = 20;
    auto burst = [&](const char *name, auto launch) {
        double issue = 0, total = 0;
        for (int r = 0; r < R + 2; r++) {
            hipStreamSynchronize(s);
            const double t0 = now_us();
            for (int i = 0; i < B; i++) launch(i);
            const double t1 = now_us();
            hipStreamSynchronize(s);
            const double t2 = now_us();
            if (r >= 2) issue += t1 - t0, total += t2 - t0;
        }
        printf("%-34s host %.3f us/launch, burst+drain %.3f us/launch\n", name, issue / (R * B), total / (R * B));
    };
    burst("hipLaunchKernelGGL grid 256", [&](int i) { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, p, i, 2, 3L); });
    burst("hipLaunchKernel (void** args)", [&](int i) {
        int a = i, b = 2; long c = 3;
        void *args[] = {&p, &a, &b, &c};
        (void)hipLaunchKernel((const void *)k_small, dim3(256), dim3(256), args, 0, s);
    });
    burst("hipExtLaunchKernel", [&](int i) {
        int a = i, b = 2; long c = 3;
        void *args[] = {&p, &a, &b, &c};
        (void)hipExtLaunchKernel((const void *)k_small, dim3(256), dim3(256), args, 0, s, nullptr, nullptr, 0);
    });
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    (void)mod;
    if (hipGetFuncBySymbol(&fn, (const void *)k_small) == hipSuccess) {
        burst("hipModuleLaunchKernel (hipFunction_t)", [&](int i) {
            int a = i, b = 2; long c = 3;
            void *args[] = {&p, &a, &b, &c};
            (void)hipModuleLaunchKernel(fn, 256, 1, 1, 256, 1, 1, 0, s, args, nullptr);
        });
    } else {
        printf("hipGetFuncBySymbol failed\n");
    }
    // graph of the same 300 launches
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
    for (int i = 0; i < B; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, p, i, 2, 3L);
    hipStreamEndCapture(s, &g);
    double t0 = now_us();
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    printf("%-34s %.1f us for %d nodes\n", "hipGraphInstantiate", now_us() - t0, B);
    size_t nn = 0;
    hipGraphGetNodes(g, nullptr, &nn);
    std::vector<hipGraphNode_t> nodes(nn);
    hipGraphGetNodes(g, nodes.data(), &nn);
    {
        double issue = 0, total = 0;
        for (int r = 0; r < R + 2; r++) {
            hipStreamSynchronize(s);
            const double a = now_us();
            hipGraphLaunch(ge, s);
            const double b = now_us();
            hipStreamSynchronize(s);
            const double c = now_us();
            if (r >= 2) issue += b - a, total += c - a;
        }
        printf("%-34s host %.3f us/kernel, launch+drain %.3f us/kernel\n", "hipGraphLaunch (300 kernels)", issue / (R * B),
               total / (R * B));
    }
    {   // update 1/3 of the nodes' arguments before every replay (n_past-dependent kernargs)
        double upd = 0, total = 0;
        for (int r = 0; r < R + 2; r++) {
            hipStreamSynchronize(s);
            const double a = now_us();
            for (size_t i = 0; i < nn; i += 3) {
                hipKernelNodeParams kp;
                hipGraphKernelNodeGetParams(nodes[i], &kp);
                int av = r, bv = 2; long cv = 3;
                void *args[] = {&p, &av, &bv, &cv};
                kp.kernelParams = args;
                hipGraphExecKernelNodeSetParams(ge, nodes[i], &kp);
            }
            const double b = now_us();
            hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            const double c = now_us();
            if (r >= 2) upd += b - a, total += c - a;
        }
        printf("%-34s %.3f us per updated node; update+replay+drain %.3f us/kernel\n", "hipGraphExecKernelNodeSetParams",
               upd / (R * ((nn + 2) / 3)), total / (R * B));
    }
    {   // capture + exec-update of a fresh capture each time (the per-eval "record" approach)
        double tot = 0;
        for (int r = 0; r < 5; r++) {
            hipStreamSynchronize(s);
            const double a = now_us();
            hipGraph_t g2;
            hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
            for (int i = 0; i < B; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, p, i + r, 2, 3L);
            hipStreamEndCapture(s, &g2);
            hipGraphNode_t err;
            hipGraphExecUpdateResult res;
            hipGraphExecUpdate(ge, g2, &err, &res);
            hipGraphLaunch(ge, s);
            const double b = now_us();
            hipStreamSynchronize(s);
            hipGraphDestroy(g2);
            tot += b - a;
            if (r == 0) printf("  exec update result %d\n", (int)res);
        }
        printf("%-34s host %.3f us/kernel (capture + exec update + launch)\n", "re-capture per eval", tot / (5 * B));
    }
    return 0;
}
