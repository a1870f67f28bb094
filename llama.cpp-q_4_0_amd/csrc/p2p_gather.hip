// p2p_gather.hip — direct-store all-gather over xGMI (the "P2P-store fallback if RCCL
// small-message latency dominates"; reference gather ggml-cuda.cu:2514-2539 copies each device's row
// slice to the main device with cudaMemcpyPeerAsync).
//
// Every rank owns a landing buffer: 2 slots x R segments x cap floats, then a flag word per peer and a
// control block.  One launch per all-gather on each rank, R - 1 workgroups: workgroup j serves peer
// q = (me + 1 + j) % R — it stores this rank's slice into segment `me` of slot (epoch & 1) of q's
// landing buffer (a plain device pointer in one process, an IPC mapping across processes), publishes
// it with a system-scope release fence and a flag store of the epoch into q's flag word `me`, then
// waits (bounded) for q's flag in its own landing buffer and copies segment q into recv.  The epoch
// lives on the device (control word 0, advanced by the last workgroup to finish), so the launch can
// be captured in a HIP graph and replayed.  Two slots suffice: peer q writes slot (e & 1) for epoch e
// only after its launch e - 1 completed, which needed this rank's e - 1 data, i.e. this rank's launch
// e - 2 (the last reader of that slot) had completed.
#include "q4_0_kernels.h"
#include "launch.h"

namespace ghip {

// Failure (a peer's flag does not arrive within a.timeout ticks of s_memrealtime, 100 MHz): the waiting
// workgroup sets its peer's bit in ctl[2] and the host-mapped error word, writes NaN into that peer's
// segment of recv instead of copying the (stale) landing slot, and NOTIFIES every peer: it ORs bit `me`
// into each peer's ctl[3] over the same mapping the data stores use (system scope).  A rank's waits poll
// its own ctl[3] beside the flag, so a peer fails within one poll of the first failure instead of
// after its own timeout (round 4: each rank paid its own 10 s on the next epoch, so an 8-rank job
// took >= 10 s per rank to error out).  ggml_hip_comm_abort sends the same notice from the host side
// (p2p_abort below; it also releases this rank's OWN gather in flight: the host sets a request word in
// host-mapped memory that the waits poll).  A comm with any bit in ctl[2] or ctl[3] is failed for good: every later launch
// only copies this rank's own slice and fills the peers' segments with NaN (no stores to peers, no
// waits, the epoch stays), and the host returns an error before launching the next all-gather
// (ggml-hip-comm.cpp comm_allgather).  Before round 4 a timed-out wait copied the stale slot and
// advanced the epoch, so the peers' epochs drifted apart and every later wait timed out in turn.
__device__ __forceinline__ void p2p_notify_peers(const P2PArgs &a) {
    for (int p = 0; p < a.R; p++)
        if (p != a.me) __hip_atomic_fetch_or(a.pctl[p] + 3, 1ull << a.me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_p2p_allgather(const P2PArgs a, const float *__restrict__ send,
                                                        int64_t count, float *__restrict__ recv) {
    const int me = a.me, R = a.R;
    const int tid = threadIdx.x;
    const uint64_t e = a.ctl[0] + 1;                 // written only by the previous launch's last workgroup
    const int slot = (int)(e & 1);
    const bool failed = __hip_atomic_load(a.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                        __hip_atomic_load(a.ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                        (a.herr && __hip_atomic_load(a.herr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0);
    const float qnan = __builtin_nanf("");
    if (blockIdx.x == 0 && recv + (int64_t)me * count != send)   // own slice (not in place)
        for (int64_t i = tid; i < count; i += blockDim.x) recv[(int64_t)me * count + i] = send[i];
    if (R > 1) {
        const int q = (me + 1 + (int)blockIdx.x) % R;
        __shared__ int s_ok;
        if (failed) {                                 // failed earlier, here or at a peer (notice)
            if (tid == 0 && a.herr) __hip_atomic_store(a.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int64_t i = tid; i < count; i += blockDim.x) recv[(int64_t)q * count + i] = qnan;
            return;
        }
        float *dst = a.land[q] + ((int64_t)slot * R + me) * a.cap;
        for (int64_t i = tid; i < count; i += blockDim.x) dst[i] = send[i];    // stores over xGMI
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");                  // system scope: the peer's view
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.flag[q] + me, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // wait for q's slice in this rank's landing buffer, bounded in time (a peer that never
            // arrives fails the comm instead of hanging the device); a peer's failure notice ends it too
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int ok = 1;
            unsigned spins = 0;
            while (__hip_atomic_load(a.flag[me] + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
                // a peer's notice (ctl[3]), another workgroup of this launch failing (ctl[2]), or this
                // rank's own abort: the host's request word (checked every 16th poll: a host-memory
                // round trip) and ctl[2] as set by k_p2p_abort on another stream
                const bool notice = __hip_atomic_load(a.ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                                    __hip_atomic_load(a.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
                const bool aborted = a.herr && (++spins & 15u) == 0 &&
                                     __hip_atomic_load(a.herr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
                const bool late = __builtin_amdgcn_s_memrealtime() - t0 > a.timeout;
                if (notice || late || aborted) {
                    __hip_atomic_fetch_or(a.ctl + 2, 1ull << q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (a.herr) __hip_atomic_store(a.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    // this rank saw the failure first (its timeout) or is the one aborting: tell the others
                    if (late || aborted) p2p_notify_peers(a);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            s_ok = ok;
        }
        __syncthreads();
        if (!s_ok) {                                  // never the stale slot: the segment reads NaN
            for (int64_t i = tid; i < count; i += blockDim.x) recv[(int64_t)q * count + i] = qnan;
            return;                                   // the epoch stays: the comm is failed
        }
        const float *src = a.land[me] + ((int64_t)slot * R + q) * a.cap;
        for (int64_t i = tid; i < count; i += blockDim.x) recv[(int64_t)q * count + i] = src[i];
    }
    // the last workgroup to finish advances the epoch for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const uint64_t old = __hip_atomic_fetch_add(a.ctl + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(a.ctl + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctl + 0, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ggml_hip_comm_abort: this rank fails (every peer bit in its own ctl[2]) and notifies every peer.  The host
// has already set herr[1], so a gather of this rank that was blocked ahead of this launch on the same stream
// has ended (and notified the peers itself) by the time this runs; on another stream, the blocked gather
// sees ctl[2] at its next poll.
__global__ void k_p2p_abort(const P2PArgs a) {
    if (threadIdx.x != 0) return;
    const uint64_t peers = (a.R >= 64 ? ~0ull : ((1ull << a.R) - 1)) & ~(1ull << a.me);
    __hip_atomic_fetch_or(a.ctl + 2, peers ? peers : 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.herr) __hip_atomic_store(a.herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    p2p_notify_peers(a);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

hipError_t p2p_abort(const P2PArgs &a, hipStream_t s) {
    if (a.R < 1 || a.R > P2P_MAX_RANKS || a.me < 0 || a.me >= a.R) return hipErrorInvalidValue;
    (void)hipGetLastError();
    launch_k(k_p2p_abort, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t p2p_allgather(const P2PArgs &a, const float *send, int64_t count, float *recv, hipStream_t s) {
    if (a.R < 1 || a.R > P2P_MAX_RANKS || a.me < 0 || a.me >= a.R || count < 0 || count > a.cap)
        return hipErrorInvalidValue;
    (void)hipGetLastError();
    launch_k(k_p2p_allgather, dim3(a.R > 1 ? a.R - 1 : 1), dim3(256), 0, s, a, send, count, recv);
    return hipGetLastError();
}

}  // namespace ghip
