// ggml-hip-graph.cpp — the launch recorder behind ghip::launch_k (launch.h).
//
// Full offload hands the backend one ggml node at a time (ggml.c:15645-15652), ~1,187 nodes and ~375
// kernel launches per decode eval of LLaMA-7B; issued one by one each launch costs ~2.6 us of host
// time (tools/host_costs2.hip), which made the end-to-end decode host bound.  While recording is on,
// launch_k appends the launch to a run; the run is submitted at the next sync point as one HIP graph:
//   * runs are keyed by their kernel sequence (function, block, LDS bytes, argument layout); a run
//     whose sequence matches a cached executable graph updates only the nodes whose grid or argument
//     bytes changed (the n_past-dependent rope / cache-copy / attention nodes of a decode eval) and
//     replays it; a new sequence is instantiated once (~1.3 ms per 48 nodes) and cached (LRU of 64);
//   * a run is submitted every GGML_HIP_GRAPH_CHUNK (48) launches, so the device overlaps the host;
//   * the nodes of a run form one dependency chain: the same order as the stream would execute them.
// The results are the kernels' own, so every bitwise test of the eager path holds for the recorded one.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "launch.h"

namespace ghip {
namespace {

constexpr int MAX_ARGS = 32;
constexpr size_t MAX_CACHED = 64;

struct Item {
    const void *fn;
    dim3 grid, block;
    size_t lds;
    int nargs;
    size_t off[MAX_ARGS];     // argument offsets in the run's blob
    size_t size[MAX_ARGS];
};

struct Run {
    std::vector<Item> items;
    std::vector<unsigned char> blob;
};

struct Cached {
    Run run;
    uint64_t sig = 0;
    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
    std::vector<hipGraphNode_t> nodes;
    hipEvent_t done = nullptr;
    uint64_t used = 0;
};

// ---- mode 2: a launcher thread.  The node walk appends each launch (function, geometry, argument
// bytes) to a ring; one worker thread issues them with hipLaunchKernel in order.  The walk's own
// logic and the ~2.6 us per hipLaunchKernel then run on two cores instead of one; every sync point
// waits until the worker has issued everything before it (same stream order as eager launches).
constexpr size_t RING = 1024, SLOT_BLOB = 1008;
struct Slot {
    const void *fn;
    int device;               // the device the launch was recorded on (the worker follows it)
    dim3 grid, block;
    uint32_t lds;
    int nargs;
    uint16_t off[MAX_ARGS];
    alignas(16) unsigned char blob[SLOT_BLOB];
};
struct Launcher {
    std::atomic<uint64_t> head{0}, tail{0};
    std::atomic<int> err{0};
    std::atomic<bool> sleeping{false};
    std::mutex mu;
    std::condition_variable cv;
    hipStream_t stream = nullptr;
    int device = 0;
    bool started = false;
    Slot ring[RING];
};
Launcher &launcher() {
    static Launcher *l = new Launcher;   // never destroyed: the worker may outlive static destructors
    return *l;
}
// the launcher's CPU: GGML_HIP_LAUNCHER_CPU=n pins it to CPU n, -1 leaves it to the scheduler; by default
// (tools/launch_thread_cost.hip: 2.75 vs 2.87 us per hipLaunchKernel pinned vs free) one of the process's own
// allowed CPUs that is neither the starting thread's nor its SMT sibling, the LOCAL_RANK-th such CPU so that
// rank processes sharing a node (and an unrestricted affinity mask) do not all spin on the same core
// (ADVICE r5); with several ranks and fewer candidate CPUs than ranks the thread stays unpinned
void launcher_pin(int main_cpu) {
    const char *e = getenv("GGML_HIP_LAUNCHER_CPU");
    const int want = e ? atoi(e) : -2;
    if (want == -1) return;
    const char *lr = getenv("LOCAL_RANK");
    const int local_rank = lr ? atoi(lr) : 0;
    cpu_set_t allowed, one;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
    int sib[2] = {-1, -1};
    char path[128];
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", main_cpu);
    if (FILE *f = fopen(path, "r")) {
        if (fscanf(f, "%d%*[,-]%d", &sib[0], &sib[1]) < 1) sib[0] = -1;
        fclose(f);
    }
    int skip = want >= 0 ? 0 : (local_rank > 0 ? local_rank : 0);
    for (int c = 0; c < CPU_SETSIZE; c++) {
        const bool ok = want >= 0 ? c == want : (CPU_ISSET(c, &allowed) && c != main_cpu && c != sib[0] && c != sib[1]);
        if (!ok || skip-- > 0) continue;
        CPU_ZERO(&one);
        CPU_SET(c, &one);
        (void)sched_setaffinity(0, sizeof one, &one);
        return;
    }
}
void launcher_main(Launcher *L, int main_cpu) {
    launcher_pin(main_cpu);
    int cur_dev = L->device;
    (void)hipSetDevice(cur_dev);
    void *argv[MAX_ARGS];
    for (;;) {
        uint64_t t = L->tail.load(std::memory_order_relaxed);
        // spin (pause, no syscalls) through an eval and the caller's ~0.7 ms between evals, then sleep:
        // (profiles/r05_e2e_launcher_spin_ab.txt: the thread mode as a whole stays box-dependent, eager is the default)
        static const long spin_us = getenv("GGML_HIP_LAUNCHER_SPIN_US") ? atol(getenv("GGML_HIP_LAUNCHER_SPIN_US")) : 2000;
        const auto t_idle = std::chrono::steady_clock::now();
        int spins = 0;
        while (L->head.load(std::memory_order_acquire) == t) {
            if ((++spins & 63) != 0 ||
                std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t_idle).count() <
                    spin_us) {
#if defined(__x86_64__)
                __builtin_ia32_pause();
#endif
                continue;
            }
            std::unique_lock<std::mutex> lk(L->mu);
            L->sleeping.store(true, std::memory_order_seq_cst);
            L->cv.wait(lk, [&] { return L->head.load(std::memory_order_acquire) != t; });
            L->sleeping.store(false, std::memory_order_relaxed);
        }
        Slot &sl = L->ring[t % RING];
        if (sl.device != cur_dev) {            // the recorded stream moved to another device
            cur_dev = sl.device;
            (void)hipSetDevice(cur_dev);
        }
        for (int a = 0; a < sl.nargs; a++) argv[a] = sl.blob + sl.off[a];
        const bool prof = g_launch_prof.load(std::memory_order_relaxed);
        const long long t0 = prof ? launch_prof_now() : 0;
        const hipError_t e = hipLaunchKernel(sl.fn, sl.grid, sl.block, argv, sl.lds, L->stream);
        if (prof) launch_prof_add(launch_prof_now() - t0);     // the worker's hipLaunchKernel cost
        if (e != hipSuccess) L->err.store((int)e, std::memory_order_relaxed);
        L->tail.store(t + 1, std::memory_order_release);
    }
}

struct Recorder {
    hipStream_t stream = nullptr;
    bool on = false;
    int mode = 1;             // 1: HIP graphs, 2: launcher thread
    Run cur;
    std::vector<Cached *> cache;
    uint64_t clock = 0;
    int ordinal = 0;          // runs submitted since the last sync point (chunk position in the eval)
    long long runs = 0, kernels = 0, updated = 0, built = 0, submit_ns = 0;
};
Recorder &rec() {
    static Recorder r;
    return r;
}
// One recorder per process, used by every thread that launches (the hook thread, loopback ranks,
// tensor-free callers): every entry point below holds this lock, so a thread's flush can never
// interleave with another thread's half-recorded run (the vector and the argument blob).
std::recursive_mutex &rec_mu() {
    static std::recursive_mutex *m = new std::recursive_mutex;   // never destroyed (atexit order)
    return *m;
}
#define REC_LOCK std::lock_guard<std::recursive_mutex> rec_lock_(rec_mu())

void fatal(hipError_t e, const char *what) {
    fprintf(stderr, "ggml-hip: launch recorder: %s failed: %s\n", what, hipGetErrorString(e));
    exit(1);
}
#define REC_CK(x)                                   \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) fatal(e_, #x);        \
    } while (0)

bool same_shape(const Item &a, const Item &b) {
    if (a.fn != b.fn || a.nargs != b.nargs || a.block.x != b.block.x || a.block.y != b.block.y ||
        a.block.z != b.block.z)
        return false;
    for (int i = 0; i < a.nargs; i++)
        if (a.size[i] != b.size[i]) return false;
    return true;
}

uint64_t signature(const Run &r, int ordinal) {
    uint64_t h = (1469598103934665603ull ^ r.items.size()) * 1099511628211ull ^ (uint64_t)ordinal;
    for (const Item &it : r.items) {
        h = (h ^ (uint64_t)(uintptr_t)it.fn) * 1099511628211ull;
        h = (h ^ (31 * it.block.x + 7 * it.nargs)) * 1099511628211ull;
    }
    return h;
}

hipKernelNodeParams params_of(Run &r, size_t i, void **argv) {
    Item &it = r.items[i];
    for (int a = 0; a < it.nargs; a++) argv[a] = r.blob.data() + it.off[a];
    hipKernelNodeParams p{};
    p.blockDim = it.block;
    p.extra = nullptr;
    p.func = const_cast<void *>(it.fn);
    p.gridDim = it.grid;
    p.kernelParams = argv;
    p.sharedMemBytes = (unsigned int)it.lds;
    return p;
}

void destroy(Cached *c) {
    if (c->done) {
        REC_CK(hipEventSynchronize(c->done));
        REC_CK(hipEventDestroy(c->done));
    }
    if (c->ex) REC_CK(hipGraphExecDestroy(c->ex));
    if (c->g) REC_CK(hipGraphDestroy(c->g));
    delete c;
}

Cached *build(Run &run, uint64_t sig) {
    Cached *c = new Cached;
    c->sig = sig;
    REC_CK(hipGraphCreate(&c->g, 0));
    c->nodes.resize(run.items.size());
    void *argv[MAX_ARGS];
    for (size_t i = 0; i < run.items.size(); i++) {
        hipKernelNodeParams p = params_of(run, i, argv);
        REC_CK(hipGraphAddKernelNode(&c->nodes[i], c->g, i ? &c->nodes[i - 1] : nullptr, i ? 1 : 0, &p));
    }
    REC_CK(hipGraphInstantiate(&c->ex, c->g, nullptr, nullptr, 0));
    REC_CK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    c->run.items.swap(run.items);
    c->run.blob.swap(run.blob);
    rec().built++;
    return c;
}

// the nodes of c whose grid or argument bytes differ from run's take run's values
// submit the pending run; chunk = the run was cut by its length (the next run continues the same
// stretch of the eval), else a sync point ends the stretch
void submit(bool chunk);

bool update(Cached *c, Run &run) {
    if (hipEventQuery(c->done) == hipErrorNotReady) REC_CK(hipEventSynchronize(c->done));
    void *argv[MAX_ARGS];
    for (size_t i = 0; i < run.items.size(); i++) {
        const Item &a = run.items[i], &b = c->run.items[i];
        bool diff = a.grid.x != b.grid.x || a.grid.y != b.grid.y || a.grid.z != b.grid.z || a.lds != b.lds;
        for (int k = 0; !diff && k < a.nargs; k++)
            diff = memcmp(run.blob.data() + a.off[k], c->run.blob.data() + b.off[k], a.size[k]) != 0;
        if (!diff) continue;
        static const bool trace = getenv("GGML_HIP_TRACE_GRAPH") && atoi(getenv("GGML_HIP_TRACE_GRAPH")) >= 2;
        if (trace) {
            int k = 0;
            while (k < a.nargs && memcmp(run.blob.data() + a.off[k], c->run.blob.data() + b.off[k], a.size[k]) == 0) k++;
            uint64_t vo = 0, vn = 0;
            if (k < a.nargs) {
                memcpy(&vo, c->run.blob.data() + b.off[k], a.size[k] < 8 ? a.size[k] : 8);
                memcpy(&vn, run.blob.data() + a.off[k], a.size[k] < 8 ? a.size[k] : 8);
            }
            fprintf(stderr, "rec_update: node %zu %s grid %u->%u lds %zu->%zu arg %d (%zu B) %llx -> %llx\n", i,
                    hipKernelNameRefByPtr(a.fn, nullptr), b.grid.x, a.grid.x, b.lds, a.lds, k, k < a.nargs ? a.size[k] : 0,
                    (unsigned long long)vo, (unsigned long long)vn);
        }
        hipKernelNodeParams p = params_of(run, i, argv);
        if (hipGraphExecKernelNodeSetParams(c->ex, c->nodes[i], &p) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        rec().updated++;
    }
    c->run.items.swap(run.items);
    c->run.blob.swap(run.blob);
    return true;
}

}  // namespace

bool rec_active(hipStream_t s) {
    REC_LOCK;
    const Recorder &r = rec();
    return r.on && s == r.stream;
}

bool rec_pending() {
    REC_LOCK;
    if (!rec().cur.items.empty() || aql_pending()) return true;
    const Launcher &L = launcher();
    return L.started && L.head.load(std::memory_order_relaxed) != L.tail.load(std::memory_order_acquire);
}

namespace {
void async_push(const void *fn, dim3 grid, dim3 block, size_t lds, int nargs, void *const *args, const size_t *sizes,
                const size_t *aligns) {
    Launcher &L = launcher();
    Recorder &r = rec();
    if (!L.started) {
        L.stream = r.stream;
        (void)hipGetDevice(&L.device);
        L.started = true;
        std::thread(launcher_main, &L, sched_getcpu()).detach();
    }
    if (L.stream != r.stream) {                // the worker serves one stream: drain, then switch
        while (L.tail.load(std::memory_order_acquire) != L.head.load(std::memory_order_relaxed)) std::this_thread::yield();
        L.stream = r.stream;
        (void)hipGetDevice(&L.device);         // the new stream's device (ggml_hip_set_main_device)
    }
    const uint64_t h = L.head.load(std::memory_order_relaxed);
    while (h - L.tail.load(std::memory_order_acquire) >= RING) std::this_thread::yield();
    Slot &sl = L.ring[h % RING];
    sl.fn = fn;
    sl.device = L.device;
    sl.grid = grid;
    sl.block = block;
    sl.lds = (uint32_t)lds;
    sl.nargs = nargs;
    size_t used = 0;
    for (int i = 0; i < nargs; i++) {
        const size_t off = (used + aligns[i] - 1) & ~(aligns[i] - 1);
        if (off + sizes[i] > SLOT_BLOB) {
            fprintf(stderr, "ggml-hip: launcher thread: %zu argument bytes exceed the slot\n", off + sizes[i]);
            exit(1);
        }
        memcpy(sl.blob + off, args[i], sizes[i]);
        sl.off[i] = (uint16_t)off;
        used = off + sizes[i];
    }
    L.head.store(h + 1, std::memory_order_release);
    if (L.sleeping.load(std::memory_order_seq_cst)) {
        std::lock_guard<std::mutex> lk(L.mu);
        L.cv.notify_one();
    }
}
void async_drain() {
    Launcher &L = launcher();
    if (!L.started) return;
    const uint64_t h = L.head.load(std::memory_order_relaxed);
    if (L.tail.load(std::memory_order_acquire) != h) {     // counted as runs / submit ns (rec_stats)
        const auto t0 = std::chrono::steady_clock::now();
        while (L.tail.load(std::memory_order_acquire) != h) std::this_thread::yield();
        rec().runs++;
        rec().submit_ns +=
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    if (const int e = L.err.exchange(0)) fatal((hipError_t)e, "hipLaunchKernel (launcher thread)");
}
}  // namespace

void rec_kernel(const void *fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, int nargs, void *const *args,
                const size_t *sizes, const size_t *aligns) {
    REC_LOCK;
    Recorder &r = rec();
    if (nargs > MAX_ARGS) {
        fprintf(stderr, "ggml-hip: launch recorder: %d kernel arguments (max %d)\n", nargs, MAX_ARGS);
        exit(1);
    }
    (void)s;
    if (r.mode == 2) {
        async_push(fn, grid, block, lds, nargs, args, sizes, aligns);
        return;
    }
    if (r.mode == 3) {
        if (aql_dispatch(fn, grid, block, lds, r.stream, nargs, args, sizes, aligns)) return;
        aql_drain();                           // the queue's work first, then this launch through HIP, in order
        aql_fallback_counted();
        REC_CK(hipLaunchKernel(fn, grid, block, const_cast<void **>(args), lds, r.stream));
        aql_stream_dirty();
        return;
    }
    Item it;
    it.fn = fn;
    it.grid = grid;
    it.block = block;
    it.lds = lds;
    it.nargs = nargs;
    for (int i = 0; i < nargs; i++) {
        size_t off = (r.cur.blob.size() + aligns[i] - 1) & ~(aligns[i] - 1);
        r.cur.blob.resize(off + sizes[i]);
        memcpy(r.cur.blob.data() + off, args[i], sizes[i]);
        it.off[i] = off;
        it.size[i] = sizes[i];
    }
    r.cur.items.push_back(it);
    // submit every `chunk` launches, so the device starts on an eval while the host still walks its
    // nodes (a whole eval as one graph would run only after the host finished: no overlap)
    static const size_t chunk = [] {
        const char *e = getenv("GGML_HIP_GRAPH_CHUNK");
        const int v = e ? atoi(e) : 0;
        return (size_t)(v > 0 ? v : 48);
    }();
    if (r.cur.items.size() >= chunk) submit(true);
}

void rec_flush_at(const char *why) {
    REC_LOCK;
    static const bool trace = getenv("GGML_HIP_TRACE_GRAPH") != nullptr;
    if (trace && rec_pending())
        fprintf(stderr, "rec_flush: %zu launches, by %s\n", rec().cur.items.size(), why);
    rec_flush();
}

void rec_flush() {
    REC_LOCK;
    async_drain();
    if (aql_pending()) aql_drain();
    aql_stream_dirty();                        // the caller's HIP call comes next (mode 3 waits for it)
    submit(false);
}

namespace {
void submit(bool chunk) {
    Recorder &r = rec();
    if (r.cur.items.empty()) return;
    const auto t0 = std::chrono::steady_clock::now();
    // runs are matched by kernel sequence AND position since the last sync point: the 32 layers of a
    // decode eval repeat one kernel sequence, and a chunk must replay its own graph (same buffers),
    // not another layer's (every node would need an update, and that graph may still be running)
    const uint64_t sig = signature(r.cur, r.ordinal);
    r.ordinal = chunk ? r.ordinal + 1 : 0;
    Cached *hit = nullptr;
    for (Cached *c : r.cache) {
        if (c->sig != sig || c->run.items.size() != r.cur.items.size()) continue;
        bool same = true;
        for (size_t i = 0; same && i < r.cur.items.size(); i++) same = same_shape(r.cur.items[i], c->run.items[i]);
        if (same) {
            hit = c;
            break;
        }
    }
    if (hit && !update(hit, r.cur)) {          // a change the executable graph cannot take: rebuild it
        for (size_t i = 0; i < r.cache.size(); i++)
            if (r.cache[i] == hit) r.cache.erase(r.cache.begin() + i);
        destroy(hit);
        hit = nullptr;
    }
    if (!hit) {
        if (r.cache.size() >= MAX_CACHED) {    // evict the least recently used
            size_t lru = 0;
            for (size_t i = 1; i < r.cache.size(); i++)
                if (r.cache[i]->used < r.cache[lru]->used) lru = i;
            destroy(r.cache[lru]);
            r.cache.erase(r.cache.begin() + lru);
        }
        hit = build(r.cur, sig);
        r.cache.push_back(hit);
    }
    hit->used = ++r.clock;
    r.runs++;
    r.kernels += (long long)hit->run.items.size();
    REC_CK(hipGraphLaunch(hit->ex, r.stream));
    REC_CK(hipEventRecord(hit->done, r.stream));
    r.cur.items.clear();
    r.cur.blob.clear();
    r.submit_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

// recording on / off for stream s; switching streams or turning recording off submits what is pending
void rec_set_mode(int mode) {
    REC_LOCK;
    rec_flush();
    rec().mode = mode == 2 || mode == 3 ? mode : 1;
}

void rec_enable(hipStream_t s, bool on) {
    REC_LOCK;
    Recorder &r = rec();
    if (s != r.stream || !on) rec_flush();
    r.stream = s;
    r.on = on;
}

void rec_stats(long long *runs, long long *kernels, long long *updated, long long *built, long long *submit_ns) {
    REC_LOCK;
    const Recorder &r = rec();
    *submit_ns = r.submit_ns;
    *runs = r.runs;
    *kernels = r.kernels;
    *updated = r.updated;
    *built = r.built;
}

std::atomic<bool> g_launch_prof{false};
std::atomic<int> g_launch_pad_ns{getenv("GGML_HIP_LAUNCH_PAD_NS") ? atoi(getenv("GGML_HIP_LAUNCH_PAD_NS")) : 0};
void launch_pad() {
    const long long until = launch_prof_now() + g_launch_pad_ns.load(std::memory_order_relaxed);
    while (launch_prof_now() < until) {}
}
static std::atomic<long long> g_lp_count{0}, g_lp_ns{0};
long long launch_prof_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void launch_prof_add(long long ns) {
    g_lp_count.fetch_add(1, std::memory_order_relaxed);
    g_lp_ns.fetch_add(ns, std::memory_order_relaxed);
}
void launch_prof_read(long long *count, long long *ns, bool reset) {
    *count = g_lp_count.load();
    *ns = g_lp_ns.load();
    if (reset) g_lp_count.store(0), g_lp_ns.store(0);
}

void rec_clear_cache() {
    REC_LOCK;
    Recorder &r = rec();
    rec_flush();
    for (Cached *c : r.cache) destroy(c);
    r.cache.clear();
}

}  // namespace ghip
