// launch_thread_cost.hip — host cost per kernel launch on the main thread vs on a launcher thread fed through a
// ring (the backend's GGML_HIP_GRAPH=2 shape), with and without pinning the worker to another core, and by API
// (hipLaunchKernel with the host stub vs hipModuleLaunchKernel with a pre-resolved hipFunction_t).
//   hipcc --offload-arch=gfx950 -O2 -pthread tools/launch_thread_cost.hip -o tools/launch_thread_cost
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <sched.h>
#include <thread>
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
    hipFunction_t fn = nullptr;
    hipGetFuncBySymbol(&fn, (const void *)k_small);
    const int B = 300, R = 20;
    cpu_set_t allowed;
    sched_getaffinity(0, sizeof allowed, &allowed);
    printf("allowed CPUs %d, main on CPU %d\n", CPU_COUNT(&allowed), sched_getcpu());
    auto launch = [&](int api, int i) {
        int a = i, b = 2;
        long c = 3;
        void *args[] = {&p, &a, &b, &c};
        if (api == 0) (void)hipLaunchKernel((const void *)k_small, dim3(256), dim3(256), args, 0, s);
        else (void)hipModuleLaunchKernel(fn, 256, 1, 1, 256, 1, 1, 0, s, args, nullptr);
    };
    for (int api = 0; api < 2; api++) {
        double issue = 0;
        for (int r = 0; r < R + 2; r++) {
            hipStreamSynchronize(s);
            const double t0 = now_us();
            for (int i = 0; i < B; i++) launch(api, i);
            if (r >= 2) issue += now_us() - t0;
        }
        printf("main thread   %-22s %.3f us/launch\n", api ? "hipModuleLaunchKernel" : "hipLaunchKernel", issue / (R * B));
    }
    // worker fed through a ring
    for (int pin = 0; pin < 2; pin++) {
        for (int api = 0; api < 2; api++) {
            std::atomic<long> head{0}, tail{0};
            std::atomic<bool> stop{false};
            std::atomic<double> wtime{0};
            const int main_cpu = sched_getcpu();
            std::thread w([&] {
                hipSetDevice(0);
                if (pin) {   // the first allowed CPU that is not the main thread's and not its SMT sibling
                    cpu_set_t one;
                    for (int c = 0; c < CPU_SETSIZE; c++) {
                        if (!CPU_ISSET(c, &allowed) || c == main_cpu) continue;
                        char path[128];
                        snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", main_cpu);
                        FILE *f = fopen(path, "r");
                        int s0 = -1, s1 = -1;
                        if (f) { if (fscanf(f, "%d%*[,-]%d", &s0, &s1) < 1) s0 = -1; fclose(f); }
                        if (c == s0 || c == s1) continue;
                        CPU_ZERO(&one);
                        CPU_SET(c, &one);
                        sched_setaffinity(0, sizeof one, &one);
                        break;
                    }
                }
                long t = 0;
                double busy = 0;
                while (!stop.load()) {
                    if (head.load(std::memory_order_acquire) == t) { std::this_thread::yield(); continue; }
                    const double t0 = now_us();
                    launch(api, (int)t);
                    busy += now_us() - t0;
                    t++;
                    tail.store(t, std::memory_order_release);
                }
                wtime.store(busy);
            });
            double total = 0;
            long pushed = 0;
            for (int r = 0; r < R + 2; r++) {
                while (tail.load() != pushed) std::this_thread::yield();
                hipStreamSynchronize(s);
                const double t0 = now_us();
                for (int i = 0; i < B; i++) head.store(++pushed, std::memory_order_release);
                while (tail.load() != pushed) std::this_thread::yield();
                if (r >= 2) total += now_us() - t0;
            }
            stop.store(true);
            w.join();
            printf("worker %-6s %-22s %.3f us/launch issued (worker busy %.3f us/launch)\n", pin ? "pinned" : "free",
                   api ? "hipModuleLaunchKernel" : "hipLaunchKernel", total / (R * B), wtime.load() / ((R + 2) * B));
        }
    }
    return 0;
}
