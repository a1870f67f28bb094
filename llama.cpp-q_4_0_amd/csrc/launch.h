// launch.h — every kernel launch of libggml_hip.so goes through ghip::launch_k.
//
// Eager by default (hipLaunchKernel).  While the launch recorder is active on the stream (full
// offload through ggml_hip_compute_forward, one device: a decode eval issues ~375 small launches
// at ~2.6 us of host time each, measured by tools/host_costs2.hip), a launch is only recorded
// (function, grid, block, LDS bytes, a copy of the argument values); the recorded run is submitted
// as one HIP graph at the next sync point (any memcpy / event / synchronize / free of the backend,
// ggml-hip-graph.cpp).  A run with the same kernels as a cached graph is submitted by updating the
// nodes whose grid or arguments changed (hipGraphExecKernelNodeSetParams, ~0.6 us per changed node)
// and one hipGraphLaunch (~0.03 us per kernel of host time).
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <new>
#include <type_traits>
#include <utility>

namespace ghip {

template <class T> struct type_tag { using type = T; };

// true while launches on s are recorded instead of issued
bool rec_active(hipStream_t s);
// launches recorded but not yet submitted
bool rec_pending();
// records one launch; args[i] points at the value of parameter i (copied before returning)
void rec_kernel(const void *fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, int nargs, void *const *args,
                const size_t *sizes, const size_t *aligns);
// submits the recorded launches (no-op when none are pending); every backend HIP call that is not
// a kernel launch calls it first (GHIP_SYNC, ggml-hip-internal.h)
void rec_flush();
void rec_flush_at(const char *why);      // the same, naming the caller (GGML_HIP_TRACE_GRAPH=1 prints it)
// recording on / off for stream s (switching stream or turning it off submits what is pending)
void rec_enable(hipStream_t s, bool on);
// 1: runs submitted as cached HIP graphs; 2: a launcher thread issues the launches in order; 3: each launch
// goes straight into an own AQL queue (ggml-hip-aql.cpp)
void rec_set_mode(int mode);
// mode 3 (ggml-hip-aql.cpp): dispatch (false: the caller launches through HIP), drain, pending, HIP-work marker
bool aql_dispatch(const void *fn, dim3 grid, dim3 block, size_t lds, hipStream_t s, int nargs, void *const *args,
                  const size_t *sizes, const size_t *aligns);
void aql_drain();
bool aql_pending();
void aql_stream_dirty();
void aql_fallback_counted();
void aql_counts(long long *out);   // dispatches, fallbacks, drains, stream syncs
// counters: submitted runs, kernels in them, nodes updated in place, graphs instantiated, host ns
// spent submitting (mode 2: waits for the launcher thread to drain, and the ns spent waiting)
void rec_stats(long long *runs, long long *kernels, long long *updated, long long *built, long long *submit_ns);
// submits what is pending and destroys every cached graph
void rec_clear_cache();
// host-cost profile of eager launches (ggml_hip_debug_launch_stats): count and ns inside hipLaunchKernel
extern std::atomic<bool> g_launch_prof;   // read by the launcher thread, written by the API
void launch_prof_add(long long ns);
long long launch_prof_now();
void launch_prof_read(long long *count, long long *ns, bool reset);
// diagnostic (GGML_HIP_LAUNCH_PAD_NS): a busy wait of this many ns after every eager launch, to measure how
// the end-to-end token time depends on the host's per-launch cost (tools/run.sh PARTS=e2e_pad)
extern std::atomic<int> g_launch_pad_ns;
void launch_pad();

template <typename... P, typename... A>
inline void launch_k(void (*k)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t s, A &&...a) {
    static_assert(sizeof...(P) == sizeof...(A), "launch_k: argument count");
    if (!rec_active(s)) {
        if (rec_pending()) rec_flush_at("eager launch");   // never overtakes recorded launches
        if (__builtin_expect(g_launch_prof.load(std::memory_order_relaxed), 0)) {
            const long long t0 = launch_prof_now();
            hipLaunchKernelGGL(k, grid, block, lds, s, std::forward<A>(a)...);
            launch_prof_add(launch_prof_now() - t0);
            return;
        }
        hipLaunchKernelGGL(k, grid, block, lds, s, std::forward<A>(a)...);
        if (__builtin_expect(g_launch_pad_ns.load(std::memory_order_relaxed) > 0, 0)) launch_pad();
        return;
    }
    // convert every argument to the parameter's exact type, then hand the recorder their addresses
    struct Holder {
        alignas(16) unsigned char raw[(sizeof(std::decay_t<P>) + ... + 0) + 16 * sizeof...(P) + 1];
    } h;
    void *ptrs[sizeof...(P) + 1];
    size_t sizes[sizeof...(P) + 1], aligns[sizeof...(P) + 1];
    size_t off = 0;
    int i = 0;
    auto put = [&](auto &&v, auto tag) {
        using T = typename decltype(tag)::type;
        static_assert(std::is_trivially_copyable<T>::value, "kernel arguments are copied bytewise");
        off = (off + alignof(T) - 1) & ~(alignof(T) - 1);
        new (h.raw + off) T(static_cast<T>(v));
        ptrs[i] = h.raw + off;
        sizes[i] = sizeof(T);
        aligns[i] = alignof(T);
        off += sizeof(T);
        i++;
    };
    (put(std::forward<A>(a), type_tag<std::decay_t<P>>{}), ...);
    rec_kernel((const void *)k, grid, block, lds, s, (int)sizeof...(P), ptrs, sizes, aligns);
}

}  // namespace ghip
