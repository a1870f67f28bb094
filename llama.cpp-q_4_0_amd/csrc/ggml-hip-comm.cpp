// ggml-hip-comm.cpp — multi-GPU (one process per GPU): communicators (RCCL, in-process loopback, file
// rendezvous), the direct-store P2P all-gather transport, and the row-split mul_mats.
#include <atomic>
#include <thread>
#include <chrono>
#include "ggml-hip-internal.h"

using namespace ghh;

#include <rccl/rccl.h>
#include <unistd.h>

// ------------------------------------------------------------------------------------------
// multi-GPU (one process per GPU) over RCCL.
//
// Transport: a communicator is either an RCCL communicator (ggml_hip_comm_init: one rank per
// process and GPU, the production path) or an in-process loopback group
// (ggml_hip_comm_init_local: R ranks driven by R host threads in ONE process, on one device or
// several).  The loopback all-gather has ncclAllGather's exact semantics (recv[r*count ...] =
// rank r's send, in place allowed, stream-ordered on every rank's stream); everything above the
// transport (the row partition, the in-place / padded-slab layouts, the compaction kernel, the
// grouped sibling all-gather) is the same code for both, so R > 1 runs on a 1-GPU box too.

namespace ghh {

struct LocalGroup {
    int R = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<const float *> send;
    std::vector<size_t> count;
    std::vector<hipEvent_t> ready, done;       // per rank: send written / copies out of it enqueued
    std::vector<double> red;                   // host all-reduce scratch [R][n]
    std::vector<std::vector<char>> blob;       // host all-gather staging (ggml_hip_comm_allgather_host)
    std::vector<void *> p2p;                   // each rank's P2P landing allocation (enable_p2p)
    std::vector<int> p2p_dev;
    int refs = 0;

    // every rank calls this with the same sequence number of collectives; blocks until all arrived
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == R) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

}  // namespace ghh

struct ggml_hip_comm {
    ncclComm_t comm = nullptr;    // RCCL, non-blocking (init and every call bounded in time, comm_settle)
    std::atomic<bool> aborted{false};   // ggml_hip_comm_abort ran: every later collective returns ERR_COMM
    LocalGroup *local = nullptr;  // loopback transport when set
    int nranks;
    int rank;
    int device;
    float *slab = nullptr;        // [nranks][N][max_rows] gather buffer
    size_t slab_bytes = 0;
    double *red_dev = nullptr;    // host-value all-reduce staging (64 doubles)
    // direct-store all-gather (ggml_hip_comm_enable_p2p, p2p_gather.hip)
    int transport = 0;            // 0: RCCL / loopback copies, 1: P2P stores
    bool p2p_on = false;
    ghip::P2PArgs p2p{};
    void *p2p_mine = nullptr;
    std::vector<void *> p2p_opened;   // IPC mappings of the peers' landing buffers
    uint32_t *p2p_herr = nullptr;     // host-mapped [0] error word (the gather sets it), [1] abort request
    double p2p_timeout_ms = -1.0;     // < 0: GGML_HIP_P2P_TIMEOUT_MS (default 10000)
    // file rendezvous transport (ggml_hip_comm_init_file): host collectives through files in fdir
    std::string fdir;
    std::string fnonce;           // this session's token: every file name carries it
    uint64_t fseq = 0;
};

namespace ghh {

#define NCCL_RET(expr)                                                                               \
    do {                                                                                             \
        ncclResult_t r_ = (expr);                                                                    \
        if (r_ != ncclSuccess) {                                                                     \
            g_last_error = std::string(#expr) + ": " + ncclGetErrorString(r_);                       \
            return GGML_HIP_ERR_COMM;                                                                \
        }                                                                                            \
    } while (0)

// RCCL bound in time (verdict r5 item 4: the first 8-GPU run must fail, not hang).  The communicator is
// non-blocking (ncclConfig_t.blocking = 0): init and every call return at once, ncclInProgress while the
// work proceeds, and comm_settle polls ncclCommGetAsyncError until it leaves that state, at most
// GGML_HIP_COMM_TIMEOUT_MS (default 120 s; init included), then aborts the communicator (ncclCommAbort)
// and fails the comm for good.  A rank that never joins init, or a peer that never enqueues its part of a
// collective's setup, thus ends in GGML_HIP_ERR_COMM on every rank that waits for it.  ggml_hip_comm_abort
// aborts it from any thread (ncclCommAbort's documented use: a collective stuck on the device).
double comm_timeout_ms() {
    const char *e = getenv("GGML_HIP_COMM_TIMEOUT_MS");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 120000.0;
}
ncclResult_t comm_settle(ggml_hip_comm *c, ncclResult_t r) {
    if (r != ncclInProgress) return r;
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = comm_timeout_ms();
    for (;;) {
        if (c->aborted.load(std::memory_order_acquire)) return ncclInvalidUsage;
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(c->comm, &st) != ncclSuccess) return ncclSystemError;
        if (st != ncclInProgress) return st;
        if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > limit) {
            if (!c->aborted.exchange(true)) (void)ncclCommAbort(c->comm);
            return ncclSystemError;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
#define NCCL_RET_C(c, expr)                                                                          \
    do {                                                                                             \
        if ((c)->aborted.load(std::memory_order_acquire)) {                                          \
            g_last_error = "RCCL communicator aborted (ggml_hip_comm_abort or a timed-out call)";    \
            return GGML_HIP_ERR_COMM;                                                                \
        }                                                                                            \
        ncclResult_t r_ = comm_settle((c), (expr));                                                  \
        if (r_ != ncclSuccess) {                                                                     \
            g_last_error = std::string(#expr) + ": " + ncclGetErrorString(r_) +                      \
                           ((c)->aborted.load() ? " (communicator aborted)" : "");                   \
            return GGML_HIP_ERR_COMM;                                                                \
        }                                                                                            \
    } while (0)

double file_timeout_s() {
    static const double limit_s = getenv("GGML_HIP_COMM_FILE_TIMEOUT_S") ? atof(getenv("GGML_HIP_COMM_FILE_TIMEOUT_S")) : 120.0;
    return limit_s;
}

// file rendezvous: rank r writes <dir>/c<nonce>_<seq>_r<r> (tmp + rename), then reads every rank's file of
// the same sequence number; a rank that sees all R files of seq knows every rank finished reading seq - 1,
// so it removes its own file of seq - 1.  Bounded wait (GGML_HIP_COMM_FILE_TIMEOUT_S, default 120 s).  The
// session nonce (file_join) keeps a reused directory from feeding a dead session's files of the same
// sequence number into this one; at most one file per rank (its last) outlives a session.
int file_allgather(ggml_hip_comm *c, const void *mine, size_t n, std::vector<char> &all) {
    const uint64_t seq = c->fseq++;
    auto name = [&](uint64_t s, int r) {
        return c->fdir + "/c" + c->fnonce + "_" + std::to_string(s) + "_r" + std::to_string(r);
    };
    const std::string me = name(seq, c->rank);
    {
        FILE *f = fopen((me + ".tmp").c_str(), "wb");
        if (!f) return fail(GGML_HIP_ERR_COMM, "file comm: cannot write " + me);
        const bool ok = fwrite(mine, 1, n, f) == n;
        if (fclose(f) != 0 || !ok) return fail(GGML_HIP_ERR_COMM, "file comm: short write " + me);
        if (rename((me + ".tmp").c_str(), me.c_str()) != 0) return fail(GGML_HIP_ERR_COMM, "file comm: rename " + me);
    }
    const double limit_s = file_timeout_s();
    all.assign(n * c->nranks, 0);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < c->nranks; r++) {
        for (;;) {
            FILE *f = fopen(name(seq, r).c_str(), "rb");
            if (f) {
                const size_t got = fread(all.data() + n * r, 1, n, f);
                fclose(f);
                if (got == n) break;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
                return fail(GGML_HIP_ERR_COMM, "file comm: timed out waiting for rank " + std::to_string(r));
            std::this_thread::sleep_for(std::chrono::microseconds(500));
        }
    }
    if (seq > 0) (void)remove(name(seq - 1, c->rank).c_str());
    return GGML_HIP_OK;
}

// The session of a file comm (collective, inside ggml_hip_comm_init_file): rank 0 publishes a fresh random
// nonce as <dir>/session with link(2), which fails when the name exists, so a directory in use or the
// leftover of a crashed session is refused loudly instead of mixing sessions; the other ranks wait for
// it (bounded), and the first all-gather of the session (the join) tells rank 0 that every rank has read
// it, after which it removes <dir>/session so the directory can host the next session.
int file_join(ggml_hip_comm *c) {
    const std::string sess = c->fdir + "/session";
    if (c->rank == 0) {
        uint64_t v = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ ((uint64_t)getpid() << 32);
        FILE *ur = fopen("/dev/urandom", "rb");
        if (ur) {
            uint64_t r = 0;
            if (fread(&r, 1, sizeof r, ur) == sizeof r) v ^= r;
            fclose(ur);
        }
        char hex[17];
        snprintf(hex, sizeof hex, "%016llx", (unsigned long long)v);
        const std::string tmp = sess + ".tmp" + hex;
        FILE *f = fopen(tmp.c_str(), "wb");
        if (!f) return fail(GGML_HIP_ERR_COMM, "file comm: cannot write " + tmp);
        const bool ok = fwrite(hex, 1, 16, f) == 16;
        if (fclose(f) != 0 || !ok) return fail(GGML_HIP_ERR_COMM, "file comm: short write " + tmp);
        const int lrc = link(tmp.c_str(), sess.c_str());
        (void)remove(tmp.c_str());
        if (lrc != 0)
            return fail(GGML_HIP_ERR_COMM, "file comm: " + sess + " exists (a session in progress, or left by a crashed "
                                           "one): use a fresh directory or remove it");
        c->fnonce = hex;
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            FILE *f = fopen(sess.c_str(), "rb");
            if (f) {
                char hex[17] = {0};
                const size_t got = fread(hex, 1, 16, f);
                fclose(f);
                if (got == 16) {
                    c->fnonce = hex;
                    break;
                }
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > file_timeout_s())
                return fail(GGML_HIP_ERR_COMM, "file comm: timed out waiting for " + sess);
            std::this_thread::sleep_for(std::chrono::microseconds(500));
        }
    }
    std::vector<char> all;
    const int32_t me = c->rank;
    const int rc = file_allgather(c, &me, sizeof me, all);   // the join: every rank has the nonce
    if (rc != GGML_HIP_OK) return rc;
    for (int r = 0; r < c->nranks; r++) {
        int32_t v;
        memcpy(&v, all.data() + sizeof v * r, sizeof v);
        if (v != r) return fail(GGML_HIP_ERR_COMM, "file comm: ranks disagree on the session");
    }
    if (c->rank == 0) (void)remove(sess.c_str());
    return GGML_HIP_OK;
}

// every rank's n bytes, in rank order, over the comm's host-side transport (RCCL through a device
// staging buffer, or files); not for loopback comms
int host_allgather_blob(ggml_hip_comm *c, const void *mine, size_t n, std::vector<char> &all) {
    if (!c->fdir.empty()) return file_allgather(c, mine, n, all);
    if (!c->comm) return fail(GGML_HIP_ERR_INVALID, "host all-gather: no RCCL or file transport");
    HIP_RET(hipSetDevice(c->device));
    char *dev = nullptr;
    HIP_RET(hipMalloc(&dev, n * c->nranks));
    all.assign(n * c->nranks, 0);
    memcpy(all.data() + n * c->rank, mine, n);
    hipStream_t s = g_dev[c->device].stream;
    int rc = GGML_HIP_OK;
    if (GHIP_SYNC(hipMemcpyAsync)(dev + n * c->rank, mine, n, hipMemcpyHostToDevice, s) != hipSuccess)
        rc = fail(GGML_HIP_ERR_DEVICE, "host all-gather: upload");
    else if (c->aborted.load() || comm_settle(c, GHIP_SYNC(ncclAllGather)(dev + n * c->rank, dev, n, ncclChar, c->comm, s)) != ncclSuccess)
        rc = fail(GGML_HIP_ERR_COMM, "host all-gather: ncclAllGather");
    else if (GHIP_SYNC(hipMemcpyAsync)(all.data(), dev, all.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
             GHIP_SYNC(hipStreamSynchronize)(s) != hipSuccess)
        rc = fail(GGML_HIP_ERR_DEVICE, "host all-gather: download");
    (void)GHIP_SYNC(hipFree)(dev);
    return rc;
}

bool p2p_failed(const ggml_hip_comm *c) {
    return c->p2p_on && c->p2p_herr && __atomic_load_n(c->p2p_herr, __ATOMIC_ACQUIRE) != 0;
}

// landing allocation of one rank: [2][R][cap] floats, then R flag words, then the control block
size_t p2p_flag_off(int R, int64_t cap) { return ((size_t)2 * R * cap * 4 + 255) & ~(size_t)255; }
size_t p2p_ctl_off(int R, int64_t cap) { return p2p_flag_off(R, cap) + 256; }
size_t p2p_bytes(int R, int64_t cap) { return p2p_ctl_off(R, cap) + 256; }

// GHIP_SYNC(ncclAllGather)(send, recv, count floats) on the comm's transport, stream-ordered on s
int comm_allgather(ggml_hip_comm *c, const float *send, float *recv, size_t count, hipStream_t s) {
    // a P2P wait that timed out failed the comm for good (its gathers fill NaN; p2p_gather.hip): the
    // error surfaces here, at the next all-gather, as the reference's CUDA_CHECK would stop at the first
    // failed copy (ggml-cuda.cu:22-51, 2514-2539)
    if (p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: the comm failed earlier (a peer wait timed out, or a rank aborted)");
    if (c->transport == 1 && c->p2p_on && (int64_t)count <= c->p2p.cap) {
        HIP_RET(ghip::p2p_allgather(c->p2p, send, (int64_t)count, recv, s));
        return GGML_HIP_OK;
    }
    if (!c->fdir.empty()) return fail(GGML_HIP_ERR_UNSUPPORTED, "file comm: device all-gathers need the P2P transport");
    if (!c->local) {
        NCCL_RET_C(c, GHIP_SYNC(ncclAllGather)(send, recv, count, ncclFloat32, c->comm, s));
        return GGML_HIP_OK;
    }
    LocalGroup &g = *c->local;
    const int me = c->rank;
    g.send[me] = send;
    g.count[me] = count;
    HIP_RET(GHIP_SYNC(hipEventRecord)(g.ready[me], s));
    g.barrier();                                             // every rank's send is published
    bool agree = true;
    for (int r = 0; r < g.R; r++) agree = agree && g.count[r] == count;
    for (int r = 0; agree && r < g.R; r++) {
        float *dst = recv + (size_t)r * count;
        if (count == 0 || (r == me && dst == send)) continue;  // in place: already there
        if (r != me) HIP_RET(GHIP_SYNC(hipStreamWaitEvent)(s, g.ready[r], 0));
        HIP_RET(GHIP_SYNC(hipMemcpyAsync)(dst, g.send[r], count * 4, hipMemcpyDefault, s));
    }
    HIP_RET(GHIP_SYNC(hipEventRecord)(g.done[me], s));
    g.barrier();                                             // every rank's copies are enqueued
    for (int r = 0; r < g.R; r++)
        if (r != me) HIP_RET(GHIP_SYNC(hipStreamWaitEvent)(s, g.done[r], 0));   // no rank reuses send early
    g.barrier();                                             // events may be re-recorded now
    return agree ? GGML_HIP_OK : fail(GGML_HIP_ERR_COMM, "loopback all-gather: ranks disagree on count");
}
int comm_group_start(ggml_hip_comm *c) {
    if (c->comm && c->transport == 0) NCCL_RET(ncclGroupStart());
    return GGML_HIP_OK;
}
int comm_group_end(ggml_hip_comm *c) {
    if (c->comm && c->transport == 0) NCCL_RET_C(c, GHIP_SYNC(ncclGroupEnd)());
    return GGML_HIP_OK;
}

}  // namespace ghh

extern "C" {

int ggml_hip_comm_unique_id(char out[GGML_HIP_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == GGML_HIP_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    NCCL_RET(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return GGML_HIP_OK;
}

int ggml_hip_comm_init(ggml_hip_comm **comm, int nranks, int rank, const char id[GGML_HIP_UNIQUE_ID_BYTES]) {
    ensure_init();
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return fail(GGML_HIP_ERR_INVALID, "bad comm arguments");
    if (nranks > ghip::SCATTER_MAX_RANKS) return fail(GGML_HIP_ERR_UNSUPPORTED, "too many ranks");
    auto *c = new (std::nothrow) ggml_hip_comm;
    if (!c) return GGML_HIP_ERR_NOMEM;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    c->nranks = nranks;
    c->rank = rank;
    c->device = current_device();
    // non-blocking init, bounded by GGML_HIP_COMM_TIMEOUT_MS (comm_settle): a rank that never joins fails
    // this one with GGML_HIP_ERR_COMM instead of hanging it
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, uid, rank, &cfg);
    if (c->comm) r = comm_settle(c, r);
    if (r != ncclSuccess) {
        if (c->comm && !c->aborted.load()) (void)ncclCommAbort(c->comm);
        delete c;
        return fail(GGML_HIP_ERR_COMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r) +
                                           " (GGML_HIP_COMM_TIMEOUT_MS bounds it)");
    }
    *comm = c;
    return GGML_HIP_OK;
}

int ggml_hip_comm_init_local(ggml_hip_comm **comms, int nranks, const int *devices) {
    ensure_init();
    if (!comms || nranks < 1 || nranks > ghip::SCATTER_MAX_RANKS) return fail(GGML_HIP_ERR_INVALID, "bad comm arguments");
    auto *g = new LocalGroup;
    g->R = nranks;
    g->send.assign(nranks, nullptr);
    g->count.assign(nranks, 0);
    g->ready.assign(nranks, nullptr);
    g->done.assign(nranks, nullptr);
    g->refs = nranks;
    const int saved = current_device();
    for (int r = 0; r < nranks; r++) {
        const int dev = devices ? devices[r] : saved;
        if (dev < 0 || dev >= g_device_count) return fail(GGML_HIP_ERR_INVALID, "bad device");
        HIP_RET(hipSetDevice(dev));
        HIP_RET(hipEventCreateWithFlags(&g->ready[r], hipEventDisableTiming));
        HIP_RET(hipEventCreateWithFlags(&g->done[r], hipEventDisableTiming));
        auto *c = new ggml_hip_comm;
        c->local = g;
        c->nranks = nranks;
        c->rank = r;
        c->device = dev;
        comms[r] = c;
    }
    HIP_RET(hipSetDevice(saved));
    return GGML_HIP_OK;
}

int ggml_hip_comm_init_file(ggml_hip_comm **comm, int nranks, int rank, const char *dir) {
    ensure_init();
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks || !dir || !*dir)
        return fail(GGML_HIP_ERR_INVALID, "bad comm arguments");
    if (nranks > ghip::SCATTER_MAX_RANKS) return fail(GGML_HIP_ERR_UNSUPPORTED, "too many ranks");
    auto *c = new (std::nothrow) ggml_hip_comm;
    if (!c) return GGML_HIP_ERR_NOMEM;
    c->nranks = nranks;
    c->rank = rank;
    c->device = current_device();
    c->fdir = dir;
    const int rc = file_join(c);
    if (rc != GGML_HIP_OK) {
        delete c;
        return rc;
    }
    *comm = c;
    return GGML_HIP_OK;
}

int ggml_hip_comm_destroy(ggml_hip_comm *c) {
    if (!c) return GGML_HIP_OK;
    if (c->p2p_on) (void)GHIP_SYNC(hipDeviceSynchronize)();
    for (void *p : c->p2p_opened) (void)hipIpcCloseMemHandle(p);
    if (c->p2p_mine) (void)GHIP_SYNC(hipFree)(c->p2p_mine);
    if (c->p2p_herr) (void)hipHostFree(c->p2p_herr);
    if (c->comm && !c->aborted.load()) ncclCommDestroy(c->comm);   // an aborted one is already freed
    if (c->slab) (void)GHIP_SYNC(hipFree)(c->slab);
    if (c->red_dev) (void)GHIP_SYNC(hipFree)(c->red_dev);
    if (c->local) {
        LocalGroup *g = c->local;
        bool last;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            last = --g->refs == 0;
        }
        if (last) {
            for (auto e : g->ready) (void)hipEventDestroy(e);
            for (auto e : g->done) (void)hipEventDestroy(e);
            delete g;
        }
    }
    delete c;
    return GGML_HIP_OK;
}

int ggml_hip_comm_allreduce_host(ggml_hip_comm *c, double *vals, int n, int op) {
    if (!c || !vals || n < 1 || n > 64 || op < 0 || op > 2) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (c->local) {
        LocalGroup &g = *c->local;
        {
            std::lock_guard<std::mutex> lk(g.mu);
            if (g.red.size() < (size_t)g.R * 64) g.red.assign((size_t)g.R * 64, 0.0);
            for (int i = 0; i < n; i++) g.red[(size_t)c->rank * 64 + i] = vals[i];
        }
        g.barrier();
        double out[64];
        {
            std::lock_guard<std::mutex> lk(g.mu);
            for (int i = 0; i < n; i++) {
                double v = g.red[i];
                for (int r = 1; r < g.R; r++) {
                    const double w = g.red[(size_t)r * 64 + i];
                    v = op == 0 ? v + w : op == 1 ? std::max(v, w) : std::min(v, w);
                }
                out[i] = v;
            }
        }
        g.barrier();
        memcpy(vals, out, sizeof(double) * n);
        return GGML_HIP_OK;
    }
    if (!c->fdir.empty()) {                   // file transport: gather every rank's values, reduce here
        std::vector<char> all;
        const int rc = file_allgather(c, vals, sizeof(double) * n, all);
        if (rc != GGML_HIP_OK) return rc;
        for (int i = 0; i < n; i++) {
            double v;
            memcpy(&v, all.data() + sizeof(double) * i, sizeof v);
            for (int r = 1; r < c->nranks; r++) {
                double w;
                memcpy(&w, all.data() + sizeof(double) * ((size_t)r * n + i), sizeof w);
                v = op == 0 ? v + w : op == 1 ? std::max(v, w) : std::min(v, w);
            }
            vals[i] = v;
        }
        return GGML_HIP_OK;
    }
    HIP_RET(hipSetDevice(c->device));
    if (!c->red_dev) HIP_RET(hipMalloc(&c->red_dev, sizeof(double) * 64));
    hipStream_t s = g_dev[c->device].stream;
    HIP_RET(GHIP_SYNC(hipMemcpyAsync)(c->red_dev, vals, sizeof(double) * n, hipMemcpyHostToDevice, s));
    const ncclRedOp_t ops[3] = {ncclSum, ncclMax, ncclMin};
    NCCL_RET_C(c, GHIP_SYNC(ncclAllReduce)(c->red_dev, c->red_dev, (size_t)n, ncclFloat64, ops[op], c->comm, s));
    HIP_RET(GHIP_SYNC(hipMemcpyAsync)(vals, c->red_dev, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_comm_allgather_host(ggml_hip_comm *c, const void *send, size_t bytes, void *recv) {
    if (!c || (!send && bytes) || (!recv && bytes)) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    std::vector<char> all;
    if (c->local) {                            // loopback: every rank's bytes through the group
        LocalGroup &g = *c->local;
        {
            std::lock_guard<std::mutex> lk(g.mu);
            if (g.blob.size() != (size_t)g.R) g.blob.assign(g.R, {});
            g.blob[c->rank].assign((const char *)send, (const char *)send + bytes);
        }
        g.barrier();
        {
            std::lock_guard<std::mutex> lk(g.mu);
            for (int r = 0; r < g.R; r++)
                if (g.blob[r].size() != bytes) {
                    g.barrier();
                    return fail(GGML_HIP_ERR_COMM, "host all-gather: ranks disagree on size");
                }
            for (int r = 0; r < g.R; r++) memcpy((char *)recv + bytes * r, g.blob[r].data(), bytes);
        }
        g.barrier();
        return GGML_HIP_OK;
    }
    const int rc = host_allgather_blob(c, send, bytes, all);
    if (rc != GGML_HIP_OK) return rc;
    memcpy(recv, all.data(), all.size());
    return GGML_HIP_OK;
}

int ggml_hip_comm_enable_p2p(ggml_hip_comm *c, int64_t max_floats) {
    ensure_init();
    if (!c || max_floats < 1) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (c->nranks > ghip::P2P_MAX_RANKS) return fail(GGML_HIP_ERR_UNSUPPORTED, "P2P all-gather: at most 8 ranks");
    if (c->p2p_on) return fail(GGML_HIP_ERR_INVALID, "P2P already enabled on this comm");
    const int R = c->nranks, me = c->rank;
    const int64_t cap = (max_floats + 63) & ~(int64_t)63;
    const size_t bytes = p2p_bytes(R, cap);
    HIP_RET(hipSetDevice(c->device));
    // Every rank takes part in every collective below whatever its local outcome (a rank that returned
    // early would leave its peers waiting in a collective); the outcomes are combined at the end, so
    // either every rank enables P2P or none does.
    int local_rc = GGML_HIP_OK;
    std::string local_msg;
    auto local_fail = [&](int rc, const std::string &m) {
        if (local_rc == GGML_HIP_OK) {
            local_rc = rc;
            local_msg = m;
        }
    };
    // fine-grained landing memory (coherent across devices); plain device memory where unavailable
    if (hipExtMallocWithFlags(&c->p2p_mine, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
        (void)hipGetLastError();
        if (hipMalloc(&c->p2p_mine, bytes) != hipSuccess) {
            c->p2p_mine = nullptr;
            local_fail(GGML_HIP_ERR_NOMEM, "P2P landing buffer");
        }
    }
    if (c->p2p_mine && (GHIP_SYNC(hipMemset)(c->p2p_mine, 0, bytes) != hipSuccess ||
                        GHIP_SYNC(hipDeviceSynchronize)() != hipSuccess))
        local_fail(GGML_HIP_ERR_DEVICE, "P2P landing buffer memset");
    // [0] error word (the gather sets it), [1] abort request (ggml_hip_comm_abort sets it, the waits poll it)
    if (hipHostMalloc((void **)&c->p2p_herr, 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        c->p2p_herr = nullptr;
        local_fail(GGML_HIP_ERR_NOMEM, "P2P host error word");
    } else {
        c->p2p_herr[0] = 0;
        c->p2p_herr[1] = 0;
    }
    uint32_t *herr_dev = nullptr;
    if (c->p2p_herr && hipHostGetDevicePointer((void **)&herr_dev, c->p2p_herr, 0) != hipSuccess)
        local_fail(GGML_HIP_ERR_DEVICE, "P2P host error word mapping");
    std::vector<char *> base(R, nullptr);
    base[me] = (char *)c->p2p_mine;
    if (c->local) {                            // one process: the peers' allocations directly
        LocalGroup &g = *c->local;
        {
            std::lock_guard<std::mutex> lk(g.mu);
            if (g.p2p.size() != (size_t)R) g.p2p.assign(R, nullptr), g.p2p_dev.assign(R, -1);
            g.p2p[me] = local_rc == GGML_HIP_OK ? c->p2p_mine : nullptr;
            g.p2p_dev[me] = c->device;
        }
        g.barrier();
        // the ranks' gathers wait on each other on the device, so the launches of ranks that share a
        // device must run concurrently; beyond two per device their streams may share a hardware queue
        // (GPU_MAX_HW_QUEUES = 4, one taken by the null stream) and a gather would wait behind a peer's.
        // Decided from the whole group's device list, so every rank takes the same decision.
        int worst = 0;
        bool all_ok = true;
        for (int r = 0; r < R; r++) {
            int same = 0;
            for (int q = 0; q < R; q++) same += g.p2p_dev[q] == g.p2p_dev[r];
            worst = std::max(worst, same);
            all_ok = all_ok && g.p2p[r] != nullptr;
        }
        if (worst > 2) local_fail(GGML_HIP_ERR_UNSUPPORTED, "loopback P2P: at most 2 ranks per device");
        else if (!all_ok) local_fail(GGML_HIP_ERR_COMM, "loopback P2P: a rank's setup failed");
        for (int r = 0; local_rc == GGML_HIP_OK && r < R; r++) {
            base[r] = (char *)g.p2p[r];
            if (g.p2p_dev[r] != c->device) {
                const hipError_t e = hipDeviceEnablePeerAccess(g.p2p_dev[r], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    local_fail(GGML_HIP_ERR_DEVICE, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();
            }
        }
        g.barrier();                           // nobody re-assigns g.p2p before all have read it
    } else {                                   // one process per GPU: IPC handles through the comm
        hipIpcMemHandle_t h;
        memset(&h, 0, sizeof h);
        static_assert(sizeof(hipIpcMemHandle_t) <= 120, "IPC handle size");
        char rec[128] = {0};                  // [0..120) the handle, [124] 1 = valid
        if (local_rc == GGML_HIP_OK) {
            const hipError_t e = hipIpcGetMemHandle(&h, c->p2p_mine);
            if (e != hipSuccess) local_fail(GGML_HIP_ERR_DEVICE, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
            else {
                memcpy(rec, &h, sizeof h);
                rec[124] = 1;
            }
        }
        std::vector<char> all;
        const int grc = host_allgather_blob(c, rec, sizeof rec, all);
        if (grc != GGML_HIP_OK) {              // the transport itself failed: no further collective can run
            const std::string msg = g_last_error;
            if (c->p2p_mine) (void)GHIP_SYNC(hipFree)(c->p2p_mine);
            c->p2p_mine = nullptr;
            if (c->p2p_herr) (void)hipHostFree(c->p2p_herr);
            c->p2p_herr = nullptr;
            return fail(grc, msg);
        }
        for (int r = 0; r < R; r++) {
            if (r == me) continue;
            if (!all[(size_t)128 * r + 124]) {
                local_fail(GGML_HIP_ERR_COMM, "P2P: rank " + std::to_string(r) + " has no IPC handle");
                continue;
            }
            if (local_rc != GGML_HIP_OK) continue;
            hipIpcMemHandle_t hr;
            memcpy(&hr, all.data() + (size_t)128 * r, sizeof hr);
            void *p = nullptr;
            const hipError_t e = hipIpcOpenMemHandle(&p, hr, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) {
                local_fail(GGML_HIP_ERR_DEVICE, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
                continue;
            }
            c->p2p_opened.push_back(p);
            base[r] = (char *)p;
        }
    }
    // every rank mapped every peer before any store, and the outcome is the group's (min over ranks)
    double v = local_rc == GGML_HIP_OK ? 1.0 : 0.0;
    const int arc = ggml_hip_comm_allreduce_host(c, &v, 1, 2);
    if (arc != GGML_HIP_OK) return arc;
    if (local_rc != GGML_HIP_OK || v < 1.0) {
        for (void *p : c->p2p_opened) (void)hipIpcCloseMemHandle(p);
        c->p2p_opened.clear();
        if (c->p2p_mine) (void)GHIP_SYNC(hipFree)(c->p2p_mine);
        c->p2p_mine = nullptr;
        if (c->p2p_herr) (void)hipHostFree(c->p2p_herr);
        c->p2p_herr = nullptr;
        if (local_rc != GGML_HIP_OK) return fail(local_rc, local_msg);
        return fail(GGML_HIP_ERR_COMM, "P2P: a peer rank's setup failed");
    }
    ghip::P2PArgs a{};
    for (int r = 0; r < R; r++) {
        a.land[r] = (float *)base[r];
        a.flag[r] = (uint64_t *)(base[r] + p2p_flag_off(R, cap));
        a.pctl[r] = (uint64_t *)(base[r] + p2p_ctl_off(R, cap));
    }
    a.ctl = (uint64_t *)((char *)c->p2p_mine + p2p_ctl_off(R, cap));
    a.herr = herr_dev;
    a.me = me;
    a.R = R;
    a.cap = cap;
    c->p2p = a;
    c->p2p_on = true;
    c->transport = 1;
    return ggml_hip_comm_set_p2p_timeout(c, c->p2p_timeout_ms);
}

int ggml_hip_comm_set_p2p_timeout(ggml_hip_comm *c, double ms) {
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null comm");
    if (ms <= 0.0) {                           // default: far above any host stall (first-call image
        const char *e = getenv("GGML_HIP_P2P_TIMEOUT_MS");   // builds, page faults, a descheduled rank)
        ms = e && atof(e) > 0.0 ? atof(e) : 10000.0;
    }
    // s_memrealtime ticks at 100 MHz; clamped so the conversion stays defined.  The timeout is
    // a kernel argument: gathers captured in a HIP graph keep the value they were captured with.
    if (!(ms < 1.0e14)) ms = 1.0e14;           // also NaN / inf
    c->p2p_timeout_ms = ms;
    c->p2p.timeout = (uint64_t)(ms * 1e5);
    return GGML_HIP_OK;
}

int ggml_hip_comm_abort(ggml_hip_comm *c) {
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null comm");
    // RCCL first (any thread): ncclCommAbort releases a collective stuck on the device, so the stream the
    // P2P notice below queues on can drain; every later call on the comm returns GGML_HIP_ERR_COMM
    if (c->comm && !c->aborted.exchange(true)) (void)ncclCommAbort(c->comm);
    if (!c->p2p_on) {
        if (c->comm) return GGML_HIP_OK;
        return fail(GGML_HIP_ERR_INVALID, "neither RCCL nor P2P on this comm");
    }
    HIP_RET(hipSetDevice(c->device));
    // first the host-mapped request word: a gather of this rank already spinning on a peer (on any stream,
    // including the one the notice below queues on) ends at its next poll and notifies the peers itself,
    // so neither this call nor the peers wait out the timeout
    if (c->p2p_herr) __atomic_store_n(c->p2p_herr + 1, 1u, __ATOMIC_RELEASE);
    hipStream_t s = g_dev[c->device].stream;
    HIP_RET(ghip::p2p_abort(c->p2p, s));
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_comm_set_transport(ggml_hip_comm *c, int transport) {
    if (!c || transport < 0 || transport > 1) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (transport == 1 && !c->p2p_on) return fail(GGML_HIP_ERR_INVALID, "P2P not enabled on this comm");
    c->transport = transport;
    return GGML_HIP_OK;
}

int ggml_hip_comm_p2p_status(ggml_hip_comm *c) {
    if (!c || !c->p2p_on) return fail(GGML_HIP_ERR_INVALID, "P2P not enabled on this comm");
    HIP_RET(hipSetDevice(c->device));
    HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());
    uint64_t err[2] = {0, 0};
    HIP_RET(GHIP_SYNC(hipMemcpy)(err, c->p2p.ctl + 2, 16, hipMemcpyDeviceToHost));
    // sticky: a failed comm stays failed.  A notice that arrived while this rank was idle (no gather of its
    // own saw it yet) is latched into the host error word here, so the next split call already returns
    // GGML_HIP_ERR_COMM instead of enqueueing one more NaN gather
    if ((err[0] | err[1]) && c->p2p_herr) __atomic_store_n(c->p2p_herr, 1u, __ATOMIC_RELEASE);
    return (int)(err[0] | err[1]);
}

int ggml_hip_comm_rank(const ggml_hip_comm *c, int *rank, int *nranks) {
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null comm");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return GGML_HIP_OK;
}

int ggml_hip_split_rows(int64_t M, int nranks, const float *tensor_split, int64_t *row_begin) {
    if (M < 0 || nranks < 1 || !row_begin) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (!tensor_split) {
        for (int r = 0; r <= nranks; r++) row_begin[r] = M * r / nranks;
        return GGML_HIP_OK;
    }
    // the reference's rule, in its float arithmetic: cumulative start fractions normalised as
    // ggml_cuda_set_tensor_split does (ggml-cuda.cu:1874-1881), then row_low = nrows0*split[id]
    // (float product truncated, ggml-cuda.cu:2363-2364) -- one routine with set_tensor_split
    if (nranks > GGML_HIP_MAX_DEVICES) return fail(GGML_HIP_ERR_INVALID, "too many ranks");
    bool all_zero = true;
    for (int r = 0; r < nranks; r++)
        if (tensor_split[r] != 0.0f) all_zero = false;
    if (all_zero) return ggml_hip_split_rows(M, nranks, nullptr, row_begin);
    float frac[GGML_HIP_MAX_DEVICES];
    split_fractions(tensor_split, nranks, frac);
    for (int r = 0; r < nranks; r++) row_begin[r] = split_row_low(M, frac, r);
    row_begin[nranks] = M;
    for (int r = 1; r <= nranks; r++)
        if (row_begin[r] < row_begin[r - 1]) row_begin[r] = row_begin[r - 1];
    return GGML_HIP_OK;
}

int ggml_hip_mul_mat_q4_0_split(ggml_hip_comm *c, const void *dev_w_local, int64_t K, int64_t M_total,
                                const int64_t *row_begin, const float *dev_x, int64_t N, float *dev_y_full,
                                void *stream) {
    if (!c || !row_begin || !dev_y_full) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: the comm failed earlier (a peer wait timed out, or a rank aborted)");
    hipStream_t s = resolve_stream(stream);
    const int R = c->nranks;
    int64_t max_rows = 0;
    bool equal = true;
    if (row_begin[0] != 0 || row_begin[R] != M_total) return fail(GGML_HIP_ERR_INVALID, "row_begin must cover [0, M)");
    for (int r = 0; r < R; r++) {
        const int64_t rows = row_begin[r + 1] - row_begin[r];
        if (rows < 0) return fail(GGML_HIP_ERR_INVALID, "row_begin must be non-decreasing");
        max_rows = std::max(max_rows, rows);
        if (rows != row_begin[1] - row_begin[0]) equal = false;
    }
    const int64_t my_rows = row_begin[c->rank + 1] - row_begin[c->rank];
    if (equal && N == 1) {
        // y_full[M] = concat of the equal rank slices: compute in place, gather in place
        float *mine = dev_y_full + row_begin[c->rank];
        if (my_rows > 0) {
            int rc = mul_mat_dev(dev_w_local, K, my_rows, dev_x, N, mine, my_rows, 0, s);
            if (rc != GGML_HIP_OK) return rc;
        }
        return comm_allgather(c, mine, dev_y_full, (size_t)my_rows, s);
    }
    // padded slabs [R][N][max_rows] -> compaction into y_full[n][M]
    const size_t slab = (size_t)N * max_rows;
    const size_t need = slab * R * 4 + slab * 4;
    if (c->slab_bytes < need) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone)
            return fail(GGML_HIP_ERR_INVALID, "split gather buffer must grow outside stream capture (run once first)");
        if (c->slab) {
            HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
            HIP_RET(GHIP_SYNC(hipFree)(c->slab));
            c->slab = nullptr;
            c->slab_bytes = 0;
        }
        HIP_RET(hipMalloc(&c->slab, need));
        c->slab_bytes = need;
    }
    float *send = c->slab + slab * R;
    if (my_rows > 0) {
        int rc = mul_mat_dev(dev_w_local, K, my_rows, dev_x, N, send, max_rows, 0, s);
        if (rc != GGML_HIP_OK) return rc;
    }
    int rc = comm_allgather(c, send, c->slab, slab, s);
    if (rc != GGML_HIP_OK) return rc;
    ghip::RowBegins rb;
    for (int r = 0; r <= R; r++) rb.v[r] = row_begin[r];
    HIP_RET(ghip::scatter_slabs(c->slab, R, max_rows, rb, N, dev_y_full, M_total, s));
    return GGML_HIP_OK;
}

int ggml_hip_mul_mat_q4_0_split_multi(ggml_hip_comm *c, int n, const void *const *dev_w_local, const int64_t *M_total,
                                      const int64_t *const *row_begin, int64_t K, const float *dev_x, int64_t N,
                                      float *const *dev_y_full, void *stream) {
    if (c && p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: the comm failed earlier (a peer wait timed out, or a rank aborted)");
    if (!c || n < 1 || n > 4 || !dev_w_local || !M_total || !row_begin || !dev_y_full)
        return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    const int R = c->nranks;
    bool equal = N == 1;
    for (int i = 0; i < n && equal; i++) {
        if (!row_begin[i] || row_begin[i][0] != 0 || row_begin[i][R] != M_total[i]) equal = false;
        for (int r = 0; r < R && equal; r++)
            if (row_begin[i][r + 1] - row_begin[i][r] != row_begin[i][1] - row_begin[i][0] ||
                row_begin[i][1] - row_begin[i][0] < 1)
                equal = false;
    }
    if (!equal) {
        for (int i = 0; i < n; i++) {
            const int rc = ggml_hip_mul_mat_q4_0_split(c, dev_w_local[i], K, M_total[i], row_begin[i], dev_x, N,
                                                       dev_y_full[i], stream);
            if (rc != GGML_HIP_OK) return rc;
        }
        return GGML_HIP_OK;
    }
    hipStream_t s = resolve_stream(stream);
    int64_t m_loc[4];
    float *mine[4];
    for (int i = 0; i < n; i++) {
        m_loc[i] = row_begin[i][c->rank + 1] - row_begin[i][c->rank];
        mine[i] = dev_y_full[i] + row_begin[i][c->rank];
    }
    int rc = ggml_hip_mul_mat_q4_0_multi(n, dev_w_local, m_loc, K, dev_x, N, mine, s);
    if (rc != GGML_HIP_OK) return rc;
    if ((rc = comm_group_start(c)) != GGML_HIP_OK) return rc;
    for (int i = 0; i < n; i++) {
        rc = comm_allgather(c, mine[i], dev_y_full[i], (size_t)m_loc[i], s);
        if (rc != GGML_HIP_OK) {
            (void)comm_group_end(c);
            return rc;
        }
    }
    return comm_group_end(c);
}

}  // extern "C"
