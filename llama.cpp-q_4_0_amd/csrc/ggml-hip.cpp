// ggml-hip.cpp — host side of the MI355X q4_0 mul_mat backend: the C ABI of include/ggml-hip.h.
//
// Mirrors the behaviour of the reference's ggml-cuda.cu host plumbing for this path
// (file:line in each function comment) with a native design:
//   * one non-blocking HIP stream per device, created once (ggml-cuda.cu:1849);
//   * a per-device caching pool for temporaries (ggml-cuda.cu:1751-1811);
//   * weights stay verbatim block_q4_0 rows in HBM (no repack), split by rows for
//     GGML_BACKEND_GPU_SPLIT (ggml-cuda.cu:2766-2809);
//   * mul_mat = fused q8_0-quantize + GEMV for N <= 8 tokens, q8_0-quantize + int8-MFMA GEMM
//     otherwise (replacing dequantize_mul_mat_vec / dequantize_block + cublasSgemm,
//     ggml-cuda.cu:1177-1244, 1156-1175, 2143-2182);
//   * multi-process multi-GPU through RCCL all-gather (no cudaMemcpy gather).
#include "../../include/ggml-hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <map>
#include <unordered_map>
#include <vector>

#include "ggml_abi.h"
#include "ggml_ops.h"
#include "q4_0_kernels.h"
#include "launch.h"

// Every HIP / RCCL call of the backend that is not a kernel launch first submits the launches the
// recorder holds (launch.h), so stream order is the order the backend issued its work in.
#define GHIP_SYNC(f) (ghip::rec_flush_at(#f " @" GHIP_STR(__LINE__)), f)
#define GHIP_STR2(x) #x
#define GHIP_STR(x) GHIP_STR2(x)

using gabi::tensor;

namespace {

constexpr int QK = 32;
constexpr int Q4B = 18;

// ------------------------------------------------------------------------------------------
// errors: the tensor ABI is fail-fast like CUDA_CHECK (ggml-cuda.cu:22-51); the tensor-free
// ABI returns a status and keeps the message for ggml_hip_last_error().

thread_local std::string g_last_error;

#define HIP_FATAL(expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "ggml-hip: HIP error %d at %s:%d: %s\n", (int)e_, __FILE__, __LINE__,     \
                    hipGetErrorString(e_));                                                          \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

#define HIP_RET(expr)                                                                                \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            g_last_error = std::string(#expr) + ": " + hipGetErrorString(e_);                        \
            return GGML_HIP_ERR_DEVICE;                                                              \
        }                                                                                            \
    } while (0)

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// ------------------------------------------------------------------------------------------
// per-device state

struct PoolBuf {
    void *ptr;
    size_t size;
};

struct Device {
    hipStream_t stream = nullptr;
    ghip::DeviceInfo info{};
    size_t total_mem = 0;
    std::mutex mu;
    std::vector<PoolBuf> pool;           // free temporaries (first-fit best size)
    void *ws = nullptr;                  // mul_mat workspace (q8_0 activations) of `stream`
    size_t ws_size = 0;
    // workspaces of other streams on this device (callers that run mul_mats on their own streams
    // concurrently, e.g. the ranks of an in-process loopback group): one per stream, never shared
    std::unordered_map<hipStream_t, PoolBuf> stream_ws;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;   // split mul_mat ordering between device streams
};

std::once_flag g_init_once;
int g_device_count = 0;
Device *g_dev = nullptr;
int g_main_device = 0;
float g_tensor_split[GGML_HIP_MAX_DEVICES] = {0};

// ggml-cuda.cu:1874-1881: cumulative start fractions in float, each divided by the float sum
static void split_fractions(const float *tensor_split, int n, float *frac) {
    float split_sum = 0.0f;
    for (int i = 0; i < n; i++) {
        frac[i] = split_sum;
        split_sum += tensor_split[i];
    }
    for (int i = 0; i < n; i++) frac[i] /= split_sum;
}

// ggml-cuda.cu:2363, 2785: row_low = nrows0*g_tensor_split[id] -- int64*float is a float product
static inline int64_t split_row_low(int64_t nrows, const float *frac, int id) {
    return id == 0 ? 0 : (int64_t)(nrows * frac[id]);
}
size_t g_scratch_size = 0;
void *g_scratch = nullptr;
size_t g_scratch_offset = 0;
bool g_eval_computed = false;            // a node ran since the last buffer assignment

void init_impl() {
    if (hipGetDeviceCount(&g_device_count) != hipSuccess) g_device_count = 0;
    if (g_device_count > GGML_HIP_MAX_DEVICES) g_device_count = GGML_HIP_MAX_DEVICES;
    g_dev = new Device[g_device_count > 0 ? g_device_count : 1];
    int cur = 0;
    if (g_device_count > 0) HIP_FATAL(hipGetDevice(&cur));
    double total = 0;
    for (int id = 0; id < g_device_count; id++) {
        hipDeviceProp_t prop;
        HIP_FATAL(hipGetDeviceProperties(&prop, id));
        g_dev[id].info.num_cus = prop.multiProcessorCount;
        g_dev[id].total_mem = prop.totalGlobalMem;
        g_tensor_split[id] = (float)total;        // default split proportional to VRAM (ggml-cuda.cu:1838-1843)
        total += (double)prop.totalGlobalMem;
        if (getenv("GGML_HIP_VERBOSE"))
            fprintf(stderr, "ggml_init_hip: device %d: %s (%s), %d CUs, %.1f GiB\n", id, prop.name,
                    prop.gcnArchName, prop.multiProcessorCount, prop.totalGlobalMem / 1073741824.0);
    }
    for (int id = 0; id < g_device_count; id++) g_tensor_split[id] = (float)(g_tensor_split[id] / total);
    for (int id = 0; id < g_device_count; id++) {
        HIP_FATAL(hipSetDevice(id));
        HIP_FATAL(hipStreamCreateWithFlags(&g_dev[id].stream, hipStreamNonBlocking));
        HIP_FATAL(hipEventCreateWithFlags(&g_dev[id].ev_a, hipEventDisableTiming));
        HIP_FATAL(hipEventCreateWithFlags(&g_dev[id].ev_b, hipEventDisableTiming));
    }
    if (g_device_count > 0) HIP_FATAL(hipSetDevice(cur));
}

inline void ensure_init() { std::call_once(g_init_once, init_impl); }

int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

hipStream_t resolve_stream(void *stream) {
    if (stream) return (hipStream_t)stream;
    ensure_init();
    return g_dev[current_device()].stream;
}

void *pool_malloc(int id, size_t size, size_t *actual) {
    Device &d = g_dev[id];
    {
        std::lock_guard<std::mutex> lk(d.mu);
        int best = -1;
        for (size_t i = 0; i < d.pool.size(); i++)
            if (d.pool[i].size >= size && (best < 0 || d.pool[i].size < d.pool[best].size)) best = (int)i;
        if (best >= 0) {
            PoolBuf b = d.pool[best];
            d.pool.erase(d.pool.begin() + best);
            *actual = b.size;
            return b.ptr;
        }
    }
    const size_t sz = (size_t)(size * 1.05) + 256;     // a little slack, like ggml_cuda_pool_malloc
    void *p = nullptr;
    HIP_FATAL(hipMalloc(&p, sz));
    *actual = sz;
    return p;
}

void pool_free(int id, void *p, size_t size) {
    Device &d = g_dev[id];
    std::lock_guard<std::mutex> lk(d.mu);
    d.pool.push_back({p, size});
}

// workspace for the q8_0 activations of one mul_mat: qs [N][K] int8 + d [N][K/32] f32 + the same d as
// fp16, block-major [K/32][N rounded up to 4] (the LDS GEMM's operand layout)
size_t ws_d16_offset(int64_t K, int64_t N) {
    const size_t qs = (size_t)(N * K + 255) & ~(size_t)255;
    return qs + (((size_t)N * (K / QK) * 4 + 255) & ~(size_t)255);
}
size_t workspace_bytes(int64_t K, int64_t N) { return ws_d16_offset(K, N) + (size_t)((N + 3) & ~3) * (K / QK) * 2; }
// the LDS GEMM (algo 2, v8 / v9) adds its x image and the per-call weight image of an M-row matrix (room
// for either image format)
size_t ws_g8x_offset(int64_t K, int64_t N) { return (workspace_bytes(K, N) + 255) & ~(size_t)255; }
size_t ws_g8w_offset(int64_t K, int64_t N) {
    return (ws_g8x_offset(K, N) + std::max(ghip::gemm8_x_bytes(K, N), ghip::gemm9_x_bytes(K, N)) + 255) & ~(size_t)255;
}
size_t workspace_bytes_mm(int64_t K, int64_t N, int64_t M) {
    return ws_g8w_offset(K, N) + std::max(ghip::gemm8_w_bytes(K, M), ghip::gemm9_w_bytes(K, M));
}
// prefill GEMM version (GGML_HIP_GEMM_V / ggml_hip_debug_set_gemm_version): 10 (default) = k_gemm9 when
// the weight has an image (ggml_hip_weight_image_create, or built on first prefill use of a
// device-resident ggml weight; images are built in fp6 format), else k_gemm7 on the q4_0 bytes; 8 = the
// same with int8 images (k_gemm8); 9 / 11 = k_gemm8 / k_gemm9 always (an unregistered weight is
// converted into the workspace per call); 7 = k_gemm7 always.  A weight's image keeps the format it
// was built in; the GEMM follows the image.
std::atomic<int> g_gemm_v{-1};
int gemm_version() {
    int v = g_gemm_v.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("GGML_HIP_GEMM_V");
        int want = e ? atoi(e) : 10, expect = -1;
        g_gemm_v.compare_exchange_strong(expect, want);
        v = g_gemm_v.load(std::memory_order_relaxed);
    }
    return v;
}

// ------------------------------------------------------------------------------------------
// int8 weight images for the prefill GEMM (k_gemm8): per device, keyed by the device
// address of the q4_0 weight.  The image is w = nibble - 8 as int8 plus the fp16 d verbatim (34 B per
// 32 weights, 1.9x the q4_0 bytes), built once by k_prep8_w; the weight must not change while an
// image of it exists (ggml weights on the device never do; every hipFree of a weight buffer here
// drops its images first).
struct WImage {
    int64_t K, M;
    void *img;
    size_t bytes;
    int fmt;                                                 // 8: int8 (k_gemm8), 9: fp6 (k_gemm9)
};
int image_format() { return gemm_version() >= 10 ? 9 : 8; }
// a weight with an image takes the image GEMM above this token count (below it the split-K GEMM on
// the q4_0 bytes; tools/n_sweep9.py: at N = 96 k_gemm9 24 / 26 / 51 us vs split-K 31 / 67 / 62 us for
// 4096^2 / 4096->11008 / 11008->4096, at N = 64 split-K still wins two of the three)
constexpr int64_t IMG_MIN_N = 64;
// ... and at any N above the GEMV's for tall matrices (4096 -> 11008: k_gemm9 23.4-24.6 us at N = 16-64
// against split-K 27.0-43.8, whose K walk streams every row per token tile)
constexpr int64_t IMG_MIN_M = 8192;
std::mutex g_wi_mu;
std::map<std::pair<int, uintptr_t>, WImage> g_wi;          // (device, weight address)
int64_t g_wi_resident = 0;

const void *wimage_find(int id, const void *w, int64_t K, int64_t M, int *fmt = nullptr) {
    std::lock_guard<std::mutex> lk(g_wi_mu);
    auto it = g_wi.find({id, (uintptr_t)w});
    if (it == g_wi.end() || it->second.K != K || it->second.M != M) return nullptr;
    if (fmt) *fmt = it->second.fmt;
    return it->second.img;
}

// build (stream-ordered on s) unless present; returns the image or nullptr on failure
const void *wimage_ensure(int id, const void *w, int64_t K, int64_t M, hipStream_t s) {
    if (const void *p = wimage_find(id, w, K, M)) return p;
    std::lock_guard<std::mutex> lk(g_wi_mu);
    auto it = g_wi.find({id, (uintptr_t)w});
    if (it != g_wi.end()) {                                  // same address, other shape: rebuild
        if (GHIP_SYNC(hipFree)(it->second.img) != hipSuccess) return nullptr;
        g_wi_resident -= (int64_t)it->second.bytes;
        g_wi.erase(it);
    }
    const int fmt = image_format();
    WImage im{K, M, nullptr, fmt == 9 ? ghip::gemm9_w_bytes(K, M) : ghip::gemm8_w_bytes(K, M), fmt};
    if (hipMalloc(&im.img, im.bytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if ((fmt == 9 ? ghip::gemm9_prep_w(w, K, M, im.img, s) : ghip::gemm8_prep_w(w, K, M, im.img, s)) != hipSuccess) {
        (void)GHIP_SYNC(hipFree)(im.img);
        return nullptr;
    }
    g_wi[{id, (uintptr_t)w}] = im;
    g_wi_resident += (int64_t)im.bytes;
    return im.img;
}

// drop the images of every weight that starts in [dev, dev + bytes) on any device (bytes == 0: at dev)
int64_t wimage_drop(const void *dev, size_t bytes) {
    const uintptr_t lo = (uintptr_t)dev, hi = lo + (bytes ? bytes : 1);
    std::lock_guard<std::mutex> lk(g_wi_mu);
    int64_t n = 0;
    for (auto it = g_wi.begin(); it != g_wi.end();) {
        if (it->first.second >= lo && it->first.second < hi) {
            HIP_FATAL(GHIP_SYNC(hipFree)(it->second.img));   // waits for kernels still reading it
            g_wi_resident -= (int64_t)it->second.bytes;
            it = g_wi.erase(it);
            n++;
        } else {
            ++it;
        }
    }
    return n;
}

int reserve_workspace(int id, size_t bytes, hipStream_t s = nullptr) {
    Device &d = g_dev[id];
    std::lock_guard<std::mutex> lk(d.mu);
    if (!s) s = d.stream;
    void *&ws = s == d.stream ? d.ws : d.stream_ws[s].ptr;
    size_t &ws_size = s == d.stream ? d.ws_size : d.stream_ws[s].size;
    if (ws_size >= bytes) return GGML_HIP_OK;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone)
        return fail(GGML_HIP_ERR_INVALID, "workspace must be reserved before stream capture");
    if (ws) {
        HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());
        HIP_RET(GHIP_SYNC(hipFree)(ws));
        ws = nullptr;
        ws_size = 0;
    }
    HIP_RET(hipMalloc(&ws, bytes));
    ws_size = bytes;
    return GGML_HIP_OK;
}

// the workspace of stream s on device id (grown on demand outside capture)
int stream_workspace(int id, hipStream_t s, size_t need, void **out) {
    Device &d = g_dev[id];
    {
        std::lock_guard<std::mutex> lk(d.mu);
        if (s == d.stream && d.ws_size >= need) {
            *out = d.ws;
            return GGML_HIP_OK;
        }
        if (s != d.stream) {
            auto it = d.stream_ws.find(s);
            if (it != d.stream_ws.end() && it->second.size >= need) {
                *out = it->second.ptr;
                return GGML_HIP_OK;
            }
        }
    }
    const int rc = reserve_workspace(id, need, s);
    if (rc != GGML_HIP_OK) return rc;
    std::lock_guard<std::mutex> lk(d.mu);
    *out = s == d.stream ? d.ws : d.stream_ws[s].ptr;
    return GGML_HIP_OK;
}

bool aligned(const void *p, size_t a) { return ((uintptr_t)p % a) == 0; }

// ------------------------------------------------------------------------------------------
// Device weight-residency cache for CPU-backend Q4_0 weights.  The arch/
// frontends never call transform_tensor, so the reference re-uploads src0 on every batched
// mul_mat (ggml-cuda.cu:2496-2502).  Here a host weight slice is uploaded once per device and
// reused while a sampled fingerprint of its bytes is unchanged (a slice rewritten in place, or a
// freed and reallocated buffer at the same address, is uploaded again).  LRU eviction under a byte
// budget (GGML_HIP_WEIGHT_CACHE_MB, default 65536); GGML_HIP_WEIGHT_CACHE=0 disables it.  Every
// tensor-ABI call ends with a stream synchronize, so an entry not used by the current call is never
// referenced by a kernel still in flight when it is evicted.

struct WCacheEntry {
    void *dev = nullptr;
    size_t bytes = 0;
    size_t img_bytes = 0;          // the prefill weight image built for this copy (counted in the budget)
    uint64_t fp = 0;
    uint64_t last_use = 0;
};
struct WCacheKey {
    const void *host;
    size_t bytes;
    int device;
    bool operator==(const WCacheKey &o) const { return host == o.host && bytes == o.bytes && device == o.device; }
};
struct WCacheHash {
    size_t operator()(const WCacheKey &k) const {
        return std::hash<const void *>()(k.host) ^ (k.bytes * 0x9E3779B97F4A7C15ull) ^ (size_t)k.device;
    }
};
std::mutex g_wc_mu;
// host copies made by ggml_hip_transform_tensor for tensors that stay on the CPU
std::mutex g_host_copy_mu;
std::unordered_map<const void *, void *> g_host_copies;
std::unordered_map<WCacheKey, WCacheEntry, WCacheHash> g_wc;
size_t g_wc_resident = 0;
uint64_t g_wc_clock = 0, g_wc_hits = 0, g_wc_misses = 0, g_wc_invalidations = 0;
std::atomic<uintptr_t> g_wc_lo{UINTPTR_MAX}, g_wc_hi{0};   // hull of the cached host ranges (monotone)

bool wcache_enabled() {
    static const bool on = !getenv("GGML_HIP_WEIGHT_CACHE") || atoi(getenv("GGML_HIP_WEIGHT_CACHE")) != 0;
    return on;
}
std::atomic<int64_t> g_decode_min_weights{-1};
int64_t decode_min_weights() {
    int64_t v = g_decode_min_weights.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("GGML_HIP_DECODE_MIN_WEIGHTS");
        v = e ? atoll(e) : (int64_t)1 << 19;
        g_decode_min_weights.store(v, std::memory_order_relaxed);
    }
    return v;
}
size_t wcache_budget() {
    static const size_t mb = getenv("GGML_HIP_WEIGHT_CACHE_MB") ? (size_t)atoll(getenv("GGML_HIP_WEIGHT_CACHE_MB")) : 65536;
    return mb << 20;
}

// GGML_HIP_WEIGHT_CACHE_VERIFY=full: fingerprint every byte on every lookup (exact, one host read of
// the weight per call); default "sampled" (below).  In-place host writes that go through ggml nodes
// are caught exactly either way (wcache_note_host_write), and ggml_hip_weight_cache_invalidate
// covers writes made outside ggml.
int wcache_verify_full() {
    static const int full = [] {
        const char *e = getenv("GGML_HIP_WEIGHT_CACHE_VERIFY");
        return e && (strcmp(e, "full") == 0 || strcmp(e, "1") == 0) ? 1 : 0;
    }();
    return full;
}
std::atomic<int> g_wc_verify_override{-1};

// every byte: 8-byte words through a multiply-xorshift chain (~10 GB/s on one core)
uint64_t wcache_fingerprint_full(const uint8_t *p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 32;
    }
    for (; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

// FNV-1a over the first and last 32 bytes and 64 evenly spaced 8-byte samples
uint64_t wcache_fingerprint(const uint8_t *p, size_t n) {
    const int ov = g_wc_verify_override.load(std::memory_order_relaxed);
    if (ov > 0 || (ov < 0 && wcache_verify_full())) return wcache_fingerprint_full(p, n);
    uint64_t h = 1469598103934665603ull ^ n;
    auto mix = [&](const uint8_t *q, size_t len) {
        for (size_t i = 0; i < len; i++) h = (h ^ q[i]) * 1099511628211ull;
    };
    mix(p, std::min<size_t>(32, n));
    if (n > 32) mix(p + n - 32, 32);
    if (n >= 64 * 8)
        for (int i = 0; i < 64; i++) mix(p + (n / 64) * (size_t)i + (n / 128), 8);
    return h;
}

// device copy of host bytes [host, host+bytes) on device id (current device = id), uploaded on
// stream s on a miss; call_id marks entries in use by the current call (never evicted by it)
const void *wcache_get(int id, const void *host, size_t bytes, hipStream_t s, uint64_t call_id) {
    const uint64_t fp = wcache_fingerprint((const uint8_t *)host, bytes);
    std::lock_guard<std::mutex> lk(g_wc_mu);
    const WCacheKey key{host, bytes, id};
    auto it = g_wc.find(key);
    if (it != g_wc.end() && it->second.fp == fp) {
        it->second.last_use = call_id;
        g_wc_hits++;
        return it->second.dev;
    }
    g_wc_misses++;
    if (it != g_wc.end()) {                                        // stale: same address, new bytes
        wimage_drop(it->second.dev, it->second.bytes);
        HIP_FATAL(GHIP_SYNC(hipFree)(it->second.dev));
        g_wc_resident -= it->second.bytes + it->second.img_bytes;
        g_wc.erase(it);
    }
    while (g_wc_resident + bytes > wcache_budget()) {             // LRU eviction
        auto victim = g_wc.end();
        for (auto e = g_wc.begin(); e != g_wc.end(); ++e)
            if (e->second.last_use != call_id && (victim == g_wc.end() || e->second.last_use < victim->second.last_use))
                victim = e;
        if (victim == g_wc.end()) break;                           // everything is in use: over budget
        wimage_drop(victim->second.dev, victim->second.bytes);
        HIP_FATAL(GHIP_SYNC(hipFree)(victim->second.dev));
        g_wc_resident -= victim->second.bytes + victim->second.img_bytes;
        g_wc.erase(victim);
    }
    WCacheEntry e;
    e.bytes = bytes;
    e.fp = fp;
    e.last_use = call_id;
    HIP_FATAL(hipMalloc(&e.dev, bytes));
    HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(e.dev, host, bytes, hipMemcpyHostToDevice, s));
    g_wc_resident += bytes;
    g_wc[key] = e;
    const uintptr_t lo = (uintptr_t)host, hi = lo + bytes;
    if (lo < g_wc_lo.load()) g_wc_lo.store(lo);
    if (hi > g_wc_hi.load()) g_wc_hi.store(hi);
    return e.dev;
}

// A prefill weight image built for a cached copy (its device address `dev`) counts against the cache
// budget with the copy and is dropped with it (images of cached copies used to sit outside the
// budget).  GGML_HIP_WEIGHT_CACHE_IMAGES=0: no images for cached copies (their prefill reads the q4_0
// bytes in place).
bool wcache_images_enabled() {
    static const bool on = !getenv("GGML_HIP_WEIGHT_CACHE_IMAGES") || atoi(getenv("GGML_HIP_WEIGHT_CACHE_IMAGES")) != 0;
    return on;
}
void wcache_note_image(int id, const void *dev, size_t img_bytes) {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    for (auto &e : g_wc)
        if (e.first.device == id && e.second.dev == dev && e.second.img_bytes == 0) {
            e.second.img_bytes = img_bytes;
            g_wc_resident += img_bytes;                // evicted from at the next miss that needs room
            return;
        }
}

// drop every cached copy whose host range overlaps [host, host + bytes) (bytes == 0: contains host);
// the next mul_mat re-uploads.  Returns the number of copies dropped.
int64_t wcache_invalidate(const void *host, size_t bytes) {
    const uintptr_t lo = (uintptr_t)host, hi = lo + (bytes ? bytes : 1);
    std::lock_guard<std::mutex> lk(g_wc_mu);
    int64_t n = 0;
    for (auto it = g_wc.begin(); it != g_wc.end();) {
        const uintptr_t a = (uintptr_t)it->first.host, b = a + it->first.bytes;
        if (a < hi && lo < b) {
            wimage_drop(it->second.dev, it->second.bytes);
            HIP_FATAL(GHIP_SYNC(hipFree)(it->second.dev));   // hipFree waits for work that still reads it
            g_wc_resident -= it->second.bytes + it->second.img_bytes;
            it = g_wc.erase(it);
            n++;
            g_wc_invalidations++;
        } else {
            ++it;
        }
    }
    return n;
}

// A ggml node about to write host memory [data, data + bytes) (every node's INIT phase, ggml.c:
// 17112-17116): cached copies of weights in that range are dropped.  This is the path of the
// reference's LoRA apply, which rewrites quantized weights in place through ggml_add_inplace /
// ggml_cpy graphs (llama.cpp:2950-2967).  One range test when nothing cached overlaps.
void wcache_note_host_write(const void *data, size_t bytes) {
    const uintptr_t lo = (uintptr_t)data, hi = lo + bytes;
    if (!data || bytes == 0 || lo >= g_wc_hi.load(std::memory_order_relaxed) ||
        hi <= g_wc_lo.load(std::memory_order_relaxed))
        return;
    wcache_invalidate(data, bytes);
}

// ------------------------------------------------------------------------------------------
// the mul_mat core (device pointers): ggml_compute_forward_mul_mat_q_f32 INIT + COMPUTE

// exact mode (algo 4 for every auto-selected mul_mat): GGML_HIP_EXACT=1 or ggml_hip_set_exact
std::atomic<int> g_exact{-1};
bool exact_mode() {
    int v = g_exact.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("GGML_HIP_EXACT");
        int want = (e && atoi(e) != 0) ? 1 : 0, expect = -1;
        g_exact.compare_exchange_strong(expect, want);
        v = g_exact.load(std::memory_order_relaxed);
    }
    return v == 1;
}

// xq: in/out mask of the q8_0(x) forms already in this stream's workspace from the previous call
// (siblings that share x: ggml_hip_mul_mat_q4_0_multi quantizes once per form): XQ_SOA = qs + d (split-K,
// exact, gemm7), XQ_G8 = the k_gemm8 x image; null = quantize; ignored by the fused GEMV
enum { XQ_SOA = 1, XQ_G8 = 2, XQ_G9 = 4 };
int mul_mat_dev(const void *w, int64_t K, int64_t M, const float *x, int64_t N, float *y, int64_t ldy, int algo,
                hipStream_t s, unsigned *xq = nullptr) {
    unsigned xq_local = 0;
    if (!xq) xq = &xq_local;
    if (!w || !x || !y || K <= 0 || M <= 0 || N < 0) return fail(GGML_HIP_ERR_INVALID, "null pointer or bad shape");
    if (N == 0) return GGML_HIP_OK;
    if (K % 64 != 0) return fail(GGML_HIP_ERR_INVALID, "K must be a multiple of 64 (ggml.c:2344 nb % 2 == 0)");
    if (ldy < M) return fail(GGML_HIP_ERR_INVALID, "ldy < M");
    if (!aligned(w, 16) || !aligned(x, 16) || !aligned(y, 4))
        return fail(GGML_HIP_ERR_INVALID, "W and x must be 16-byte aligned, y 4-byte aligned");
    if (M * (K / QK) * Q4B >= ((int64_t)1 << 31) || N * K >= ((int64_t)1 << 31) || M >= (1 << 30))
        return fail(GGML_HIP_ERR_UNSUPPORTED, "matrix too large for 32-bit buffer offsets; split rows");
    const int id = current_device();
    const int max_nt = ghip::gemv_max_tokens(K);
    // auto: exact mode if switched on; else fused GEMV for N <= 8, split-K MFMA for N <= 128,
    // LDS-staged MFMA GEMM above (crossovers measured with tools/n_sweep.py); a
    // weight with an image takes the image GEMM from N > IMG_MIN_N (tools/n_sweep9.py)
    if (algo == 0) {
        if (exact_mode()) algo = 4;
        else if (N <= max_nt) algo = 1;
        else if (N > 128) algo = 2;
        else if ((N > IMG_MIN_N || M >= IMG_MIN_M) && gemm_version() >= 8 && wimage_find(id, w, K, M)) algo = 2;
        else algo = 3;
    }
    if (algo == 1) {
        if (N > max_nt) return fail(GGML_HIP_ERR_INVALID, "GEMV path supports N <= gemv_max_tokens(K)");
        HIP_RET(ghip::gemv_q4_0(w, K, M, x, N, y, ldy, g_dev[id].info, s));
        return GGML_HIP_OK;
    }
    if (algo < 2 || algo > 4) return fail(GGML_HIP_ERR_INVALID, "algo must be 0, 1, 2, 3 or 4");
    void *ws = nullptr;
    const int gv = gemm_version();
    int fmt = 0;
    const void *wimg = algo == 2 && gv >= 8 ? wimage_find(id, w, K, M, &fmt) : nullptr;
    if (algo == 2 && (wimg || gv == 9 || gv == 11)) {   // k_gemm8 / k_gemm9 on weight + x images
        if (!wimg) fmt = gv == 11 ? 9 : 8;
        const int wrc = stream_workspace(id, s, workspace_bytes_mm(K, N, wimg ? 0 : M), &ws);
        if (wrc != GGML_HIP_OK) return wrc;
        void *xws = (char *)ws + ws_g8x_offset(K, N);
        const unsigned form = fmt == 9 ? XQ_G9 : XQ_G8;        // one x image region: the forms exclude
        if (!(*xq & form))
            HIP_RET(fmt == 9 ? ghip::gemm9_prep_x(x, K, N, xws, s) : ghip::gemm8_prep_x(x, K, N, xws, s));
        *xq = (*xq & ~(unsigned)(XQ_G8 | XQ_G9)) | form;
        if (!wimg) {                            // unregistered weight: converted per call
            void *wws = (char *)ws + ws_g8w_offset(K, N);
            HIP_RET(fmt == 9 ? ghip::gemm9_prep_w(w, K, M, wws, s) : ghip::gemm8_prep_w(w, K, M, wws, s));
            wimg = wws;
        }
        HIP_RET(fmt == 9 ? ghip::gemm9_run(wimg, K, M, xws, N, y, ldy, s) : ghip::gemm8_run(wimg, K, M, xws, N, y, ldy, s));
        return GGML_HIP_OK;
    }
    const int wrc = stream_workspace(id, s, workspace_bytes(K, N), &ws);
    if (wrc != GGML_HIP_OK) return wrc;
    int8_t *qs = (int8_t *)ws;
    float *xd = (float *)((char *)ws + ((size_t)(N * K + 255) & ~(size_t)255));
    uint16_t *xd16 = (uint16_t *)((char *)ws + ws_d16_offset(K, N));
    // the fp16 block-major d_x copy (gemm7) is written whenever qs/d are: a sibling group may mix algos
    if (!(*xq & XQ_SOA)) HIP_RET(ghip::quantize_q8_0_soa(x, K, N, qs, xd, s, xd16));
    *xq |= XQ_SOA;
    if (algo == 4)
        HIP_RET(ghip::mm_exact_q4_0(w, K, M, qs, xd, N, y, ldy, s));
    else if (algo == 3)
        HIP_RET(ghip::gemm_sk_q4_0(w, K, M, qs, xd, N, y, ldy, g_dev[id].info.num_cus, s));
    else
        HIP_RET(ghip::gemm_q4_0(w, K, M, qs, xd, N, y, ldy, s, xd16));
    return GGML_HIP_OK;
}

// Sibling matrices (one x) that all take k_gemm9 on a registered fp6 image: ONE launch over their
// row tiles (the x image built once, as before).  Each output is computed exactly as by the
// per-matrix launch (same block order, same workgroup-half split), so y is bitwise the same.
// Returns 1 when the group does not qualify (the caller runs one launch per matrix).
int mul_mat_group_g9(int n, const void *const *w, const int64_t *M, int64_t K, const float *x, int64_t N,
                     float *const *y, hipStream_t s) {
    static const bool grp = !getenv("GGML_HIP_GEMM9_GROUP") || atoi(getenv("GGML_HIP_GEMM9_GROUP")) != 0;
    const int gv = gemm_version();
    if (!grp || n < 2 || n > 4 || gv != 10 || !x || K <= 0 || K % 64 != 0 || !aligned(x, 16) ||
        N <= ghip::gemv_max_tokens(K) || N * K >= ((int64_t)1 << 31))
        return 1;
    const int id = current_device();
    const void *img[4];
    int64_t ldy[4];
    for (int i = 0; i < n; i++) {
        int fmt = 0;
        img[i] = wimage_find(id, w[i], K, M[i], &fmt);
        // mul_mat_dev's algo rule: the image GEMM above 128 tokens, or above IMG_MIN_N / for tall
        // matrices when an image exists
        if (!img[i] || fmt != 9 || !(N > 128 || N > IMG_MIN_N || M[i] >= IMG_MIN_M)) return 1;
        if (M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31) || M[i] >= (1 << 30)) return 1;
        ldy[i] = M[i];
    }
    void *ws = nullptr;
    const int wrc = stream_workspace(id, s, workspace_bytes_mm(K, N, 0), &ws);
    if (wrc != GGML_HIP_OK) return wrc;
    void *xws = (char *)ws + ws_g8x_offset(K, N);
    HIP_RET(ghip::gemm9_prep_x(x, K, N, xws, s));
    HIP_RET(ghip::gemm9_run_multi(n, img, M, K, xws, N, y, ldy, s));
    return GGML_HIP_OK;
}

// ------------------------------------------------------------------------------------------
// tensor helpers

bool is_contiguous(const tensor *t) {
    const size_t ts = gabi::type_size(t->type);
    const int bs = gabi::blck_size(t->type);
    return t->nb[0] == ts && t->nb[1] == t->nb[0] * t->ne[0] / bs && t->nb[2] == t->nb[1] * t->ne[1] &&
           t->nb[3] == t->nb[2] * t->ne[2];
}

bool on_device(const tensor *t) {
    return t && (t->backend == gabi::BACKEND_GPU || t->backend == gabi::BACKEND_GPU_SPLIT);
}

void split_range(int64_t nrows, int id, int64_t *lo, int64_t *hi) {
    // ggml-cuda.cu:2361-2368 / 2779-2786
    *lo = split_row_low(nrows, g_tensor_split, id);
    *hi = id == g_device_count - 1 ? nrows : split_row_low(nrows, g_tensor_split, id + 1);
}

bool supported_mul_mat(const tensor *src0, const tensor *src1, const tensor *dst) {
    return src0 && src1 && dst && src0->type == gabi::TYPE_Q4_0 && src1->type == gabi::TYPE_F32 &&
           dst->type == gabi::TYPE_F32 && src0->ne[0] % 64 == 0 && src0->ne[0] == src1->ne[0] &&
           dst->ne[0] == src0->ne[1] && dst->ne[1] == src1->ne[1] && src0->ne[2] == src1->ne[2] &&
           src0->ne[3] == src1->ne[3] && is_contiguous(src0) && is_contiguous(src1) && is_contiguous(dst);
}

[[noreturn]] void op_abort(const tensor *t, const char *why) {
    // the reference asserts the same way (GGML_ASSERT in ggml-cuda.cu's op wrappers): a node that
    // reaches a device op must be computable there, ggml.c cannot fall back once an operand is on
    // the device (ggml.c:15650)
    fprintf(stderr, "ggml_hip_compute_forward: op %d (%s): %s\n", t->op, t->name, why);
    abort();
}

// ------------------------------------------------------------------------------------------
// device storage of graph tensors (assign_buffers) and of uploaded tensors

std::mutex g_own_mu;
std::unordered_map<void *, int> g_owned;                 // hipMalloc'ed by this backend for a tensor
std::unordered_map<const tensor *, ggml_tensor_extra_gpu *> g_graph_extra;   // reused across evals

void own_device_buffer(void *p) {
    std::lock_guard<std::mutex> lk(g_own_mu);
    g_owned[p] = 1;
}
bool release_device_buffer(void *p) {      // true when p was allocated by this backend (free it)
    std::lock_guard<std::mutex> lk(g_own_mu);
    return g_owned.erase(p) != 0;
}
void forget_graph_extra(const tensor *t, ggml_tensor_extra_gpu *extra) {
    std::lock_guard<std::mutex> lk(g_own_mu);
    auto it = g_graph_extra.find(t);
    if (it != g_graph_extra.end() && it->second == extra) g_graph_extra.erase(it);
    delete extra;
}

// ggml-cuda.cu:2830-2892.  Graph tensors of an eval live in a context that is reset every eval, at
// the same addresses: their extras are kept per tensor address and reused (the reference leaks one
// per offloaded node per eval).
void assign_buffers_impl(tensor *t, bool scratch, bool force_inplace) {
    if (scratch && g_scratch_size == 0) return;
    ensure_init();
    if (g_device_count == 0) return;
    // recursively assign buffers until a compute tensor is found
    if (t->src0 && t->src0->backend == gabi::BACKEND_CPU) {
        const int op0 = t->src0->op;
        if (op0 == gabi::OP_RESHAPE || op0 == gabi::OP_TRANSPOSE || op0 == gabi::OP_VIEW)
            assign_buffers_impl(t->src0, scratch, force_inplace);
    }
    if (t->op == gabi::OP_CPY && t->src1->backend == gabi::BACKEND_CPU) assign_buffers_impl(t->src1, scratch, force_inplace);

    t->backend = gabi::BACKEND_GPU;
    ggml_tensor_extra_gpu *extra;
    {
        std::lock_guard<std::mutex> lk(g_own_mu);
        auto it = g_graph_extra.find(t);
        if (it == g_graph_extra.end()) it = g_graph_extra.emplace(t, new ggml_tensor_extra_gpu).first;
        extra = it->second;
    }
    memset(extra, 0, sizeof(*extra));
    const bool inplace = (t->src0 && t->src0->data == t->data) || t->op == gabi::OP_VIEW || force_inplace;
    const size_t size = gabi::nbytes(t);
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    if (inplace && t->src0 && on_device(t->src0)) {
        size_t offset = 0;
        if (t->op == gabi::OP_VIEW) memcpy(&offset, t->opt[0]->data, sizeof(size_t));   // ggml_view_impl
        extra->data_device[id] = (char *)((ggml_tensor_extra_gpu *)t->src0->extra)->data_device[id] + offset;
    } else if (t->op == gabi::OP_CPY) {
        extra->data_device[id] = ((ggml_tensor_extra_gpu *)t->src1->extra)->data_device[id];
    } else if (scratch) {
        if (size > g_scratch_size) {
            fprintf(stderr, "ggml_hip_assign_buffers: tensor of %zu bytes exceeds the %zu-byte scratch\n", size,
                    g_scratch_size);
            abort();
        }
        if (g_scratch_offset + size > g_scratch_size) g_scratch_offset = 0;
        if (!g_scratch) HIP_FATAL(hipMalloc(&g_scratch, g_scratch_size));
        extra->data_device[id] = (char *)g_scratch + g_scratch_offset;
        // slots rounded up to 64 KiB (smaller for a small scratch: at most 1/2048 of it, at least 256 B;
        // kernels load 16 B): the attention tensors of a decode eval grow by one key per token (KQ:
        // 128 B per token at 32 heads), and with coarse slots the nodes after them keep their addresses
        // from eval to eval (launch recorder, launch.h)
        size_t gran = 65536;
        while (gran > 256 && gran > g_scratch_size / 2048) gran >>= 1;
        g_scratch_offset += (size + gran - 1) & ~(gran - 1);
    } else {
        void *p = nullptr;
        HIP_FATAL(hipMalloc(&p, size ? size : 1));
        HIP_FATAL(GHIP_SYNC(hipMemset)(p, 0, size));
        own_device_buffer(p);
        extra->data_device[id] = p;
    }
    t->extra = extra;
}

// ------------------------------------------------------------------------------------------
// host-built lookup tables of the CPU ops (bit-exact restatements, ggml_ops.hip)

uint16_t f32_to_f16_bits(float f) {          // GGML_FP32_TO_FP16 (F16C _cvtss_sh(x, 0): RNE)
    const _Float16 h = (_Float16)f;
    uint16_t b;
    memcpy(&b, &h, 2);
    return b;
}
float f16_bits_to_f32(uint16_t b) {
    _Float16 h;
    memcpy(&h, &b, 2);
    return (float)h;
}

struct OpTables {
    uint16_t *silu = nullptr;                // table_silu_f16 (ggml.c:4252)
    uint16_t *exp = nullptr;                 // table_exp_f16  (ggml.c:4253)
};
std::mutex g_tab_mu;
OpTables g_tabs[GGML_HIP_MAX_DEVICES];

// ggml_init builds them as fp16(silu(f)) and fp16(expf(f)) for every fp16 bit pattern f with the
// host libm (ggml.c:4246-4254); the same formula with the same libm gives the same 2 x 64 K entries
const OpTables &op_tables(int id, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    OpTables &t = g_tabs[id];
    if (!t.silu) {
        std::vector<uint16_t> silu(65536), ex(65536);
#pragma clang loop vectorize(disable)
        for (int i = 0; i < 65536; i++) {
            const float f = f16_bits_to_f32((uint16_t)i);
            silu[i] = f32_to_f16_bits(f / (1.0f + expf(-f)));
            ex[i] = f32_to_f16_bits(expf(f));
        }
        HIP_FATAL(hipMalloc(&t.silu, 2 * 65536 * sizeof(uint16_t)));
        t.exp = t.silu + 65536;
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(t.silu, silu.data(), 65536 * 2, hipMemcpyHostToDevice, s));
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(t.exp, ex.data(), 65536 * 2, hipMemcpyHostToDevice, s));
        HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    }
    return t;
}

// rope (mode 0) cos/sin per position p and pair j of a row of ne0 values: theta starts at (float)p
// and is multiplied by theta_scale = powf(10000.0, -2.0f/n_dims) once per pair, cos/sin by the host
// libm (ggml.c:12772, 12811-12816).  One table per (ne0, n_dims), grown to the positions seen.
struct RopeTable {
    int64_t ne0 = 0;
    int n_dims = 0;
    int64_t npos = 0;
    float *dev = nullptr;                    // float2 [npos][ne0/2]
};
std::vector<RopeTable> g_rope[GGML_HIP_MAX_DEVICES];

const float *rope_table(int id, int64_t ne0, int n_dims, int64_t need_pos, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    RopeTable *rt = nullptr;
    for (auto &r : g_rope[id])
        if (r.ne0 == ne0 && r.n_dims == n_dims) rt = &r;
    if (!rt) {
        g_rope[id].push_back(RopeTable{});
        rt = &g_rope[id].back();
        rt->ne0 = ne0;
        rt->n_dims = n_dims;
    }
    if (rt->npos < need_pos) {
        int64_t npos = std::max<int64_t>(need_pos, 2 * rt->npos);
        npos = std::max<int64_t>(npos, 512);
        const int64_t np = ne0 / 2;
        const float theta_scale = powf(10000.0, -2.0f / n_dims);
        std::vector<float> h((size_t)(npos * np * 2));
        for (int64_t p = 0; p < npos; p++) {
            float theta = (float)p;
            for (int64_t j = 0; j < np; j++) {
                h[(size_t)(p * np + j) * 2] = cosf(theta);
                h[(size_t)(p * np + j) * 2 + 1] = sinf(theta);
                theta *= theta_scale;
            }
        }
        if (rt->dev) {
            HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));   // earlier ropes may still read the old table
            HIP_FATAL(GHIP_SYNC(hipFree)(rt->dev));
        }
        HIP_FATAL(hipMalloc(&rt->dev, h.size() * sizeof(float)));
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(rt->dev, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, s));
        HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
        rt->npos = npos;
    }
    return rt->dev;
}

// ------------------------------------------------------------------------------------------
// the non-Q4_0 device ops (ggml-cuda.cu:2569-2760 + ggml_cuda_op 2286-2567, restated): operands on
// the device are used in place, host operands are staged through pool temporaries, a host dst is
// downloaded; a node whose operands are all device resident is only enqueued (no synchronize)

struct OpCall {
    int id;
    hipStream_t s;
    std::vector<std::pair<void *, size_t>> tmp;
    bool sync = false;
    void *temp(size_t bytes) {
        size_t a = 0;
        void *p = pool_malloc(id, bytes ? bytes : 16, &a);
        tmp.push_back({p, a});
        return p;
    }
    // device address of t's data (host tensors uploaded; they must be contiguous)
    char *in(const tensor *t) {
        if (t->backend == gabi::BACKEND_GPU) return (char *)((ggml_tensor_extra_gpu *)t->extra)->data_device[id];
        if (t->backend == gabi::BACKEND_GPU_SPLIT) op_abort(t, "row-split operand outside a Q4_0 mul_mat");
        if (!is_contiguous(t)) op_abort(t, "non-contiguous host operand of a device op");
        const size_t bytes = gabi::nbytes(t);
        void *p = temp(bytes);
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(p, t->data, bytes, hipMemcpyHostToDevice, s));
        sync = true;
        return (char *)p;
    }
    char *out(const tensor *t) {
        if (t->backend == gabi::BACKEND_GPU) return (char *)((ggml_tensor_extra_gpu *)t->extra)->data_device[id];
        if (!is_contiguous(t)) op_abort(t, "non-contiguous host destination of a device op");
        sync = true;
        return (char *)temp(gabi::nbytes(t));
    }
    void finish(const tensor *dst, const char *d) {
        if (dst->backend != gabi::BACKEND_GPU)
            HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(dst->data, d, gabi::nbytes(dst), hipMemcpyDeviceToHost, s));
        if (sync) HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
        for (auto &x : tmp) pool_free(id, x.first, x.second);
    }
};

bool same_shape(const tensor *a, const tensor *b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}

std::atomic<int64_t> g_op_count[gabi::OP_COUNT];      // device nodes run, per ggml op (debug stats)
std::atomic<int64_t> g_host_ns{0};                     // host time inside the taken nodes (debug stats)
std::atomic<int64_t> g_op_ns[gabi::OP_COUNT];          // the same, per op of the node that arrived
// fused launches by chain: add/rms_norm/mul, scale/mask/soft_max, silu/mul, rope/cpy, KQV/merge cpy,
// q4_0 mul_mat run under a pending silu, sibling q4_0 GEMVs (wq|wk|wv, w1|w3) run as one group,
// independent rope / rope->cpy / cpy nodes held behind a group run as one launch, the decode
// soft_max chain with its KQV and merged copy as one launch
// soft_max chain with its KQV and merged copy as one launch, the decode norm / silu chains in the GEMV
// prologue (9, 10), the prefill chains that wrote the k_gemm9 x image of their output (11)
constexpr int N_FUSED = 12;
std::atomic<int64_t> g_fused[N_FUSED];

// fused_cpy: a CPY node consuming t (rope -> cpy into the K cache; f16 mul_mat -> permute(0,2,1,3)
// -> contiguous cpy), checked by try_fuse; its destination is written by t's own kernel
void run_device_op(tensor *t, const tensor *fused_cpy = nullptr) {
    const int op = t->op;
    if (op >= 0 && op < gabi::OP_COUNT) g_op_count[op].fetch_add(1, std::memory_order_relaxed);
    if (op == gabi::OP_RESHAPE || op == gabi::OP_VIEW || op == gabi::OP_PERMUTE || op == gabi::OP_TRANSPOSE) return;
    const tensor *a = t->src0, *b = t->src1;
    OpCall c{g_main_device, nullptr, {}};
    HIP_FATAL(hipSetDevice(c.id));
    c.s = g_dev[c.id].stream;
    auto f32 = [&](const tensor *x) {
        if (x->type != gabi::TYPE_F32) op_abort(t, "operand type must be F32");
    };
    switch (op) {
        case gabi::OP_ADD: {                                     // ggml.c:8260
            f32(a), f32(b), f32(t);
            if (!same_shape(a, b) || !same_shape(a, t) || !is_contiguous(a) || !is_contiguous(b) || !is_contiguous(t))
                op_abort(t, "add needs contiguous operands of one shape");
            const char *pa = c.in(a), *pb = c.in(b);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_add_f32((const float *)pa, (const float *)pb, (float *)d,
                                       t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3], c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_MUL: {                                     // ggml.c:9149 (rows of b repeat)
            f32(a), f32(b), f32(t);
            if (!same_shape(a, t) || b->ne[0] != a->ne[0] || a->ne[1] % b->ne[1] || a->ne[2] % b->ne[2] ||
                a->ne[3] % b->ne[3] || !is_contiguous(a) || !is_contiguous(b) || !is_contiguous(t))
                op_abort(t, "mul needs contiguous operands, b rows repeating over a");
            const char *pa = c.in(a), *pb = c.in(b);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_mul_f32((const float *)pa, (const float *)pb, (float *)d, a->ne[0], a->ne[1], a->ne[2],
                                       a->ne[3], b->ne[1], b->ne[2], b->ne[3], c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_SILU: {                                    // ggml.c:10188 (GGML_SILU_FP16)
            f32(a), f32(t);
            if (!same_shape(a, t) || !is_contiguous(a) || !is_contiguous(t)) op_abort(t, "silu needs contiguous operands");
            const OpTables &tb = op_tables(c.id, c.s);
            const char *pa = c.in(a);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_silu_f32((const float *)pa, (float *)d, t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3],
                                        tb.silu, c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_RMS_NORM: {                                // ggml.c:10389
            f32(a), f32(t);
            if (!same_shape(a, t) || !is_contiguous(a) || !is_contiguous(t)) op_abort(t, "rms_norm needs contiguous rows");
            const char *pa = c.in(a);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_rms_norm_f32((const float *)pa, (float *)d, a->ne[0], gabi::nrows(a), a->ne[0], t->ne[0],
                                            c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_SCALE: {                                   // ggml.c:11633, scale factor read on the host
            f32(a), f32(t);
            if (!same_shape(a, t) || !is_contiguous(a) || !is_contiguous(t) || b->backend != gabi::BACKEND_CPU)
                op_abort(t, "scale needs contiguous operands and a host scalar");
            const float v = *(const float *)b->data;
            const char *pa = c.in(a);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_scale_f32((const float *)pa, (float *)d, v, t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3], c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_DIAG_MASK_INF: {                           // ggml.c:12195
            f32(a), f32(t);
            if (!same_shape(a, t) || !is_contiguous(a) || !is_contiguous(t) || b->backend != gabi::BACKEND_CPU)
                op_abort(t, "diag_mask_inf needs contiguous operands and host parameters");
            const int n_past = ((const int32_t *)b->data)[0];
            const char *pa = c.in(a);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_diag_mask_inf_f32((const float *)pa, (float *)d, a->ne[0], gabi::nrows(a), a->ne[1], n_past,
                                                 c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_SOFT_MAX: {                                // ggml.c:12284
            f32(a), f32(t);
            if (!same_shape(a, t) || !is_contiguous(a) || !is_contiguous(t)) op_abort(t, "soft_max needs contiguous rows");
            const OpTables &tb = op_tables(c.id, c.s);
            const char *pa = c.in(a);
            char *d = c.out(t);
            HIP_FATAL(ghip::op_soft_max_f32((const float *)pa, (float *)d, a->ne[0], gabi::nrows(a), tb.exp, c.s));
            c.finish(t, d);
            return;
        }
        case gabi::OP_ROPE: {                                    // ggml.c:12714, mode 0 (LLaMA)
            f32(a), f32(t);
            if (b->backend != gabi::BACKEND_CPU) op_abort(t, "rope parameters must be a host tensor");
            const int n_past = ((const int32_t *)b->data)[0];
            const int n_dims = ((const int32_t *)b->data)[1];
            const int mode = ((const int32_t *)b->data)[2];
            if (mode != 0) op_abort(t, "only rope mode 0 is implemented on the device");
            if (!same_shape(a, t) || a->nb[0] != 4 || t->nb[0] != 4 || a->ne[0] % 2 || n_dims % 2 || n_past < 0)
                op_abort(t, "rope needs f32 rows of even length");
            const int64_t np = a->ne[0] / 2;
            const float *cs = rope_table(c.id, a->ne[0], n_dims, (int64_t)n_past + a->ne[2], c.s);
            const char *pa = c.in(a);
            char *d = c.out(t);
            // a host source was uploaded contiguous: its strides are the contiguous ones
            int64_t nbx[4], nbd[4];
            for (int i = 0; i < 4; i++) {
                nbx[i] = a->backend == gabi::BACKEND_GPU ? (int64_t)a->nb[i] : 0;
                nbd[i] = t->backend == gabi::BACKEND_GPU ? (int64_t)t->nb[i] : 0;
            }
            if (a->backend != gabi::BACKEND_GPU) nbx[1] = a->ne[0] * 4, nbx[2] = nbx[1] * a->ne[1], nbx[3] = nbx[2] * a->ne[2];
            if (t->backend != gabi::BACKEND_GPU) nbd[1] = t->ne[0] * 4, nbd[2] = nbd[1] * t->ne[1], nbd[3] = nbd[2] * t->ne[2];
            if (fused_cpy) {
                const tensor *cb = fused_cpy->src1;
                HIP_FATAL(ghip::op_rope_cpy_f32(pa, d, a->ne, nbx, nbd, cs + (size_t)n_past * np * 2, (int)np,
                                                (char *)((ggml_tensor_extra_gpu *)cb->extra)->data_device[c.id],
                                                cb->type == gabi::TYPE_F16, cb->ne[0], cb->ne[1], cb->nb[0], cb->nb[1],
                                                cb->nb[2], c.s));
            } else {
                HIP_FATAL(ghip::op_rope_f32(pa, d, a->ne, nbx, nbd, cs + (size_t)n_past * np * 2, (int)np, c.s));
            }
            c.finish(t, d);
            return;
        }
        case gabi::OP_CPY: {                                     // ggml-cuda.cu:2690-2727: src0 -> src1 (a view)
            if (a->type != gabi::TYPE_F32 || (b->type != gabi::TYPE_F32 && b->type != gabi::TYPE_F16))
                op_abort(t, "cpy supports F32 -> F32 / F16");
            if (a->backend != gabi::BACKEND_GPU || b->backend != gabi::BACKEND_GPU)
                op_abort(t, "cpy needs both operands on the device (ggml-cuda.cu:2695-2696)");
            if (a->ne[3] != 1 || b->ne[3] != 1) op_abort(t, "cpy supports 3-d tensors");
            const int64_t n = a->ne[0] * a->ne[1] * a->ne[2];
            if (n != b->ne[0] * b->ne[1] * b->ne[2]) op_abort(t, "cpy element counts differ");
            const char *pa = c.in(a);
            char *pb = (char *)((ggml_tensor_extra_gpu *)b->extra)->data_device[c.id];
            HIP_FATAL(ghip::op_cpy_f32(pa, pb, b->type == gabi::TYPE_F16, n, a->ne[0], a->ne[1], a->nb[0], a->nb[1],
                                       a->nb[2], b->ne[0], b->ne[1], b->nb[0], b->nb[1], b->nb[2], c.s));
            c.finish(b, pb);
            return;
        }
        case gabi::OP_MUL_MAT: {                                 // F16 x F32: ggml.c:11026 (attention on the KV cache)
            if (b->type != gabi::TYPE_F32 || t->type != gabi::TYPE_F32 || a->nb[0] != 2 || b->nb[0] != 4)
                op_abort(t, "f16 mul_mat needs F16 rows (nb00 = 2) x F32 rows (nb10 = 4) -> F32");
            if (a->backend != gabi::BACKEND_GPU) op_abort(t, "f16 mul_mat needs src0 on the device");
            if (a->ne[0] != b->ne[0] || a->ne[2] != b->ne[2] || a->ne[3] != 1 || b->ne[3] != 1 || t->ne[0] != a->ne[1] ||
                t->ne[1] != b->ne[1] || t->ne[2] != a->ne[2] || !is_contiguous(t))
                op_abort(t, "f16 mul_mat shape");
            if (a->ne[0] > INT32_MAX) op_abort(t, "f16 mul_mat K too large");
            const char *pa = c.in(a);
            const char *pb = c.in(b);
            int64_t nb11 = b->nb[1], nb12 = b->nb[2];
            if (b->backend != gabi::BACKEND_GPU) nb11 = b->ne[0] * 4, nb12 = nb11 * b->ne[1];
            char *d = c.out(t);
            float *merged =
                fused_cpy ? (float *)((ggml_tensor_extra_gpu *)fused_cpy->src1->extra)->data_device[c.id] : nullptr;
            // fast mode: the many-row (prefill) products on the matrix cores; exact mode: the AVX chains bit for bit
            HIP_FATAL(ghip::op_mul_mat_f16_f32(pa, pb, (float *)d, (int)a->ne[0], a->ne[1], b->ne[1], a->ne[2], a->nb[1],
                                               a->nb[2], nb11, nb12, c.s, merged, exact_mode() ? -1 : -2));
            c.finish(t, d);
            return;
        }
        default:
            op_abort(t, "not a device op");
    }
}

// ------------------------------------------------------------------------------------------
// Launch fusion of back-to-back full-offload nodes.  A decode token is ~830 dependent launches of
// ~2.6 us host cost each (tools/host_costs.hip), so chains that ggml emits one after the other are
// run as one kernel: add -> rms_norm -> mul(norm weight), rms_norm -> mul, scale -> diag_mask_inf
// -> soft_max, silu ... mul (across the one q4_0 mul_mat between them), rope -> cpy (into the K
// cache) and the f16 mul_mat KQV -> permute(0,2,1,3) -> contiguous cpy.  The producer node is
// deferred until its consumer arrives; anything else flushes it first, and so does every other
// backend entry point (its output is device memory, observable only through the backend).  The
// fused kernels store every intermediate tensor as its own node would, bit for bit.
// GGML_HIP_FUSE=0 runs every node as its own launch.

// GGML_HIP_NORM_FOLD: 1 (default) the decode norm chains and silu -> mul run in the consuming GEMVs' x
// prologue, 2 the norm chains only, 0 neither (each chain its own launch)
std::atomic<int> g_norm_fold{-1};
int norm_fold_mode() {
    int v = g_norm_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = getenv("GGML_HIP_NORM_FOLD") ? atoi(getenv("GGML_HIP_NORM_FOLD")) : 1;
        v = v < 0 || v > 2 ? 1 : v;
        g_norm_fold.store(v, std::memory_order_relaxed);
    }
    return v;
}
bool norm_fold_enabled() { return norm_fold_mode() != 0; }
bool silu_fold_enabled() { return norm_fold_mode() == 1; }

// GGML_HIP_X9_FOLD=0: a prefill norm / silu chain whose consumers all take k_gemm9 runs as its own
// launch and the mul_mats build the x image themselves (k_prep9_x); on (default), the chain's kernel
// writes the image beside its f32 output
std::atomic<int> g_x9_fold{-1};
bool x9_fold_enabled() {
    int v = g_x9_fold.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_X9_FOLD") || atoi(getenv("GGML_HIP_X9_FOLD")) != 0) ? 1 : 0;
        g_x9_fold.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

std::atomic<int> g_fuse{-1};
bool fuse_enabled() {
    int v = g_fuse.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_FUSE") || atoi(getenv("GGML_HIP_FUSE")) != 0) ? 1 : 0;
        g_fuse.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

// ---- held-node snapshots (graph lifetime).  A held node (pending chain, group member, node held
// behind a group) can outlive its ggml_graph_compute: a caller may end a graph on a device-only node
// and ggml_free the context before the next backend call flushes it.  Every node is therefore copied
// when it is held, with its operands two levels deep, into a backend-owned arena; the copies carry
// everything a deferred launch reads (shapes, strides, extras, the host scalar parameters of scale /
// rope / diag_mask_inf), and flushes run on the copies only.  Identity tests against an arriving
// node (t->src0 == held) compare the original address AND the original's fields at hold time, so a
// new graph that reuses a freed address never fuses with a stale node.
struct SnapTensor {
    tensor t;                  // working copy: src0 / src1 -> copies, host parameters -> param
    const tensor *orig = nullptr;
    tensor pristine;           // the original's bytes when it was copied
    int depth = -1;
    alignas(16) uint8_t param[16];
};
constexpr size_t SNAP_BLOCK = 1024;
struct SnapArena {
    std::vector<std::unique_ptr<SnapTensor[]>> blocks;     // stable addresses
    size_t used = 0;
    std::unordered_map<const tensor *, SnapTensor *> memo;  // original -> copy
};
SnapArena g_snaps;

bool is_snap(const tensor *t) {
    for (const auto &b : g_snaps.blocks)
        if ((const char *)t >= (const char *)b.get() && (const char *)t < (const char *)(b.get() + SNAP_BLOCK)) return true;
    return false;
}
// the fields a graph does not change after building it (n_tasks and the perf counters excluded)
bool stable_equal(const tensor *a, const tensor *b) {
    return memcmp(a, b, offsetof(tensor, n_tasks)) == 0 &&
           memcmp(&a->data, &b->data, offsetof(tensor, padding) - offsetof(tensor, data)) == 0;
}
tensor *snap(tensor *t, int depth) {
    if (!t || is_snap(t)) return t;
    auto it = g_snaps.memo.find(t);
    SnapTensor *c = nullptr;
    if (it != g_snaps.memo.end() && stable_equal(t, &it->second->pristine)) {
        c = it->second;
        if (c->depth >= depth) return &c->t;
    } else {                   // new, or a freed address reused by another tensor: a fresh copy
        const size_t bi = g_snaps.used / SNAP_BLOCK;
        if (bi == g_snaps.blocks.size()) g_snaps.blocks.emplace_back(new SnapTensor[SNAP_BLOCK]);
        c = &g_snaps.blocks[bi][g_snaps.used % SNAP_BLOCK];
        g_snaps.used++;
        c->t = *t;
        c->pristine = *t;
        c->orig = t;
        c->t.grad = nullptr;
        for (int i = 0; i < gabi::MAX_OPT; i++) c->t.opt[i] = nullptr;
        c->t.src0 = c->t.src1 = nullptr;
        if (t->backend == gabi::BACKEND_CPU && t->data && (t->type == gabi::TYPE_F32 || t->type == gabi::TYPE_I32) &&
            gabi::nbytes(t) <= sizeof(c->param)) {
            memcpy(c->param, t->data, gabi::nbytes(t));
            c->t.data = c->param;
        }
        g_snaps.memo[t] = c;
    }
    c->depth = depth;
    if (depth > 0) {           // t is the live original here: it is being held right now
        c->t.src0 = snap(t->src0, depth - 1);
        c->t.src1 = snap(t->src1, depth - 1);
    }
    return &c->t;
}
tensor *hold(tensor *t) { return snap(t, 2); }
void snap_reset() {
    g_snaps.used = 0;
    g_snaps.memo.clear();
}
// is x (arriving, or a copy) the tensor h (a held copy)?
bool same_tensor(const tensor *x, const tensor *h) {
    if (x == h) return true;
    if (!x || !h) return false;
    const bool sx = is_snap(x), sh = is_snap(h);
    if (sx == sh) return false;            // two copies (one per tensor) or two live originals
    const SnapTensor *c = (const SnapTensor *)(sh ? h : x);
    const tensor *o = sh ? x : h;
    return o == c->orig && stable_equal(o, &c->pristine);
}

struct Pending {
    int n = 0;
    tensor *node[4] = {};
};
Pending g_pend;

// ---- a completed chain of one row (decode) that produces the src1 of q4_0 mul_mats, held for them:
// they run it in their x prologue (ghip::gemv_q4_0_multi_norm), one launch less per chain; anything
// else runs it as its own launch.  kind 1: [add ->] rms_norm -> mul (op_add_rms_norm_mul_f32; out =
// the mul), kind 2: silu -> mul (op_silu_mul_f32; a = the silu input, b = the mul's other operand,
// norm = the silu output)
struct NormChain {
    bool on = false;
    int kind = 1;
    int nn = 0;
    tensor *node[3] = {};          // held copies of the chain's nodes (for the counters)
    tensor *out_node = nullptr;    // the chain's last node (its output is the GEMVs' src1)
    const float *a = nullptr, *b = nullptr, *w = nullptr;
    float *sum = nullptr, *norm = nullptr, *out = nullptr;
    const uint16_t *table = nullptr;
    int64_t ncols = 0;
    int64_t nrows = 1;             // > 1: a prefill chain held for q4_0 mul_mats on fp6 images (x image fold)
};
NormChain g_norm;
void mul_mat_node(const tensor *src0, const tensor *src1, tensor *dst);

char *dptr(const tensor *t) { return (char *)((ggml_tensor_extra_gpu *)t->extra)->data_device[g_main_device]; }
bool dev_f32(const tensor *t) {
    return t && t->backend == gabi::BACKEND_GPU && t->type == gabi::TYPE_F32 && t->extra && is_contiguous(t);
}
bool host_scalar_param(const tensor *t) { return t && t->backend == gabi::BACKEND_CPU && t->data; }
bool overlaps(const tensor *a, const tensor *b) {   // device byte ranges of two device tensors
    if (!a || !b || a->backend != gabi::BACKEND_GPU || b->backend != gabi::BACKEND_GPU || !a->extra || !b->extra) return false;
    const char *pa = dptr(a), *pb = dptr(b);
    return pa < pb + gabi::nbytes(b) && pb < pa + gabi::nbytes(a);
}

bool deferrable(const tensor *t) {
    if (!fuse_enabled() || !dev_f32(t)) return false;
    switch (t->op) {
        case gabi::OP_ADD:
            return dev_f32(t->src0) && dev_f32(t->src1) && same_shape(t, t->src0) && same_shape(t, t->src1);
        case gabi::OP_RMS_NORM:
        case gabi::OP_SILU:
            return dev_f32(t->src0) && same_shape(t, t->src0);
        case gabi::OP_SCALE:
            return dev_f32(t->src0) && same_shape(t, t->src0) && host_scalar_param(t->src1);
        case gabi::OP_ROPE:
            return dev_f32(t->src0) && same_shape(t, t->src0) && t->ne[3] == 1 && host_scalar_param(t->src1) &&
                   ((const int32_t *)t->src1->data)[2] == 0;
        case gabi::OP_MUL_MAT:       // f16 x f32 (attention): the consumer may be the KQV merge copy
            return t->src0 && t->src0->type == gabi::TYPE_F16 && t->src0->backend == gabi::BACKEND_GPU && t->src1 &&
                   t->src1->type == gabi::TYPE_F32 && t->src1->backend == gabi::BACKEND_GPU && t->src1->extra;
        default:
            return false;
    }
}

void count_node(const tensor *t) { g_op_count[t->op].fetch_add(1, std::memory_order_relaxed); }

// the pending scale -> diag_mask_inf -> soft_max chain (nodes 0..2 of p) in one launch
void launch_softmax_chain(const Pending &p) {
    const tensor *sc = p.node[0], *mk = p.node[1], *t = p.node[2];
    const int id = g_main_device;
    hipStream_t s = g_dev[id].stream;
    const OpTables &tb = op_tables(id, s);
    float *d = (float *)dptr(t);
    HIP_FATAL(hipSetDevice(id));
    HIP_FATAL(ghip::op_scale_mask_soft_max_f32((const float *)dptr(sc->src0), dptr(sc) == (char *)d ? nullptr : (float *)dptr(sc),
                                               dptr(mk) == (char *)d ? nullptr : (float *)dptr(mk), d,
                                               *(const float *)sc->src1->data, t->ne[0], gabi::nrows(t), t->ne[1],
                                               ((const int32_t *)mk->src1->data)[0], tb.exp, s));
    for (int i = 0; i < 3; i++) count_node(p.node[i]);
    g_fused[1].fetch_add(1, std::memory_order_relaxed);
}
bool softmax_chain(const Pending &p) {
    return p.n >= 3 && p.node[0]->op == gabi::OP_SCALE && p.node[1]->op == gabi::OP_DIAG_MASK_INF &&
           p.node[2]->op == gabi::OP_SOFT_MAX;
}

void flush_pending() {
    const Pending p = g_pend;
    g_pend = Pending{};
    int i = 0;
    if (softmax_chain(p)) {             // held lazily for a possible KQV: complete it as one launch
        launch_softmax_chain(p);
        i = 3;
    }
    for (; i < p.n; i++) run_device_op(p.node[i]);
}

bool dev_overlap(const tensor *a, const tensor *b);
size_t span_bytes(const tensor *t);

// a chain of nrows rows that may be held for the k_gemm9 x image fold
bool x9_chain_ok(int64_t ncols, int64_t nrows) {
    return x9_fold_enabled() && !exact_mode() && gemm_version() == 10 && nrows > IMG_MIN_N && ghip::op_x9_ok(ncols, nrows) &&
           nrows * ncols < ((int64_t)1 << 31);
}

// t arrives while a chain is pending: extend the chain, complete it in one launch, or let a q4_0
// mul_mat that touches none of its buffers run first.  false: t does not fit (caller flushes).
bool try_fuse(tensor *t) {
    Pending &p = g_pend;
    tensor *last = p.node[p.n - 1];
    const int id = g_main_device;
    hipStream_t s = g_dev[id].stream;
    // add -> rms_norm(sum): extend
    if (p.n == 1 && last->op == gabi::OP_ADD && t->op == gabi::OP_RMS_NORM && same_tensor(t->src0, last) && deferrable(t)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // scale -> diag_mask_inf(scaled): extend
    if (p.n == 1 && last->op == gabi::OP_SCALE && t->op == gabi::OP_DIAG_MASK_INF && same_tensor(t->src0, last) && dev_f32(t) &&
        same_shape(t, last) && host_scalar_param(t->src1)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // [add ->] rms_norm -> mul(norm weight row): complete
    if (last->op == gabi::OP_RMS_NORM && t->op == gabi::OP_MUL && same_tensor(t->src0, last) && dev_f32(t) && same_shape(t, last) &&
        dev_f32(t->src1) && t->src1->ne[0] == t->ne[0] && t->src1->ne[1] == 1 && t->src1->ne[2] == 1 && t->src1->ne[3] == 1) {
        const tensor *add = p.n == 2 ? p.node[0] : nullptr;
        const tensor *x = add ? add : last->src0;     // the rms_norm input
        // one row (decode): hold it for the q4_0 GEMVs that follow (norm_fold)
        NormChain c;
        c.a = add ? (const float *)dptr(add->src0) : nullptr;
        c.b = add ? (const float *)dptr(add->src1) : (const float *)dptr(x);
        c.sum = add ? (float *)dptr(add) : nullptr;
        c.norm = (float *)dptr(last);
        c.w = (const float *)dptr(t->src1);
        c.out = (float *)dptr(t);
        c.ncols = t->ne[0];
        auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
        bool fold = norm_fold_enabled() && !exact_mode() && gabi::nrows(t) == 1 && c.ncols % 64 == 0 &&
                    c.ncols <= 16384 && al(c.a) && al(c.b) && al(c.sum) && al(c.norm) && al(c.w) && al(c.out);
        // the chain's outputs must not alias its inputs (the GEMV's workgroups read the inputs while
        // workgroup 0 stores the outputs)
        for (const tensor *o : {add, (const tensor *)last, (const tensor *)t})
            for (const tensor *i : {(const tensor *)(add ? add->src0 : nullptr), (const tensor *)(add ? add->src1 : x),
                                    (const tensor *)t->src1})
                if (o && i && dev_overlap(o, i)) fold = false;
        // many rows (prefill): hold it too; if the q4_0 mul_mats that consume it all take k_gemm9, its
        // launch writes their x image (flush_group_x9), else it runs as below when they flush it
        if (x9_chain_ok(c.ncols, gabi::nrows(t)) && al(c.a) && al(c.b) && al(c.sum) && al(c.norm) && al(c.w) && al(c.out)) {
            fold = true;
            c.nrows = gabi::nrows(t);
        }
        if (fold) {
            for (int i = 0; i < p.n; i++) c.node[c.nn++] = p.node[i];
            c.node[c.nn++] = hold(t);
            c.out_node = c.node[c.nn - 1];
            c.on = true;
            g_norm = c;
            p = Pending{};
            return true;
        }
        HIP_FATAL(hipSetDevice(id));
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32(add ? (const float *)dptr(add->src0) : nullptr,
                                                add ? (const float *)dptr(add->src1) : (const float *)dptr(x),
                                                add ? (float *)dptr(add) : nullptr, (float *)dptr(last),
                                                (const float *)dptr(t->src1), (float *)dptr(t), t->ne[0], gabi::nrows(t), s));
        for (int i = 0; i < p.n; i++) count_node(p.node[i]);
        count_node(t);
        g_fused[0].fetch_add(1, std::memory_order_relaxed);
        p = Pending{};
        return true;
    }
    // scale -> diag_mask_inf -> soft_max: held (completed as one launch by flush_pending, or with
    // the KQV that follows at decode)
    if (p.n == 2 && p.node[0]->op == gabi::OP_SCALE && last->op == gabi::OP_DIAG_MASK_INF && t->op == gabi::OP_SOFT_MAX &&
        same_tensor(t->src0, last) && dev_f32(t) && same_shape(t, last)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // soft_max chain -> KQV (f16 V^T . softmax, one query row per head): extend
    if (p.n == 3 && softmax_chain(p) && t->op == gabi::OP_MUL_MAT && same_tensor(t->src1, last) && t->src0 &&
        t->src0->type == gabi::TYPE_F16 && t->src0->backend == gabi::BACKEND_GPU && t->src0->extra &&
        t->src0->nb[0] == 2 && t->src0->ne[3] == 1 && last->ne[1] == 1 && last->ne[3] == 1 &&
        t->src0->ne[0] == last->ne[0] && t->src0->ne[2] == last->ne[2] && last->ne[0] <= 16384 && dev_f32(t) &&
        t->ne[1] == 1 && t->ne[0] == t->src0->ne[1] && dev_f32(p.node[0]->src0)) {
        p.node[p.n++] = hold(t);
        return true;
    }
    // soft_max chain -> KQV -> cpy(permute(KQV)) (the merged heads): complete as one launch
    if (p.n == 4 && softmax_chain(p) && t->op == gabi::OP_CPY && t->src0 && t->src0->op == gabi::OP_PERMUTE &&
        same_tensor(t->src0->src0, last)) {
        const tensor *m = t->src0, *cb = t->src1;
        if (m->ne[0] == last->ne[0] && m->ne[1] == last->ne[2] && m->ne[2] == last->ne[1] && m->ne[3] == 1 &&
            m->nb[0] == 4 && m->nb[1] == last->nb[2] && m->nb[2] == last->nb[1] && dev_f32(cb) &&
            gabi::nbytes(cb) == gabi::nbytes(last) && !overlaps(cb, last) && !overlaps(cb, last->src0) &&
            !overlaps(cb, p.node[2]) && !overlaps(cb, p.node[0]->src0)) {
            const tensor *sc = p.node[0], *mk = p.node[1], *sm = p.node[2], *kqv = last, *vv = kqv->src0;
            const char *kq = dptr(sc->src0);
            // stores into the buffer the workgroups read (the in-place chain) are skipped: see
            // k_softmax_kqv; no node reads them, KQV consumes the softmax inside the launch
            auto out = [&](const tensor *x) { return overlaps(x, sc->src0) ? nullptr : (float *)dptr(x); };
            const OpTables &tb = op_tables(id, s);
            HIP_FATAL(hipSetDevice(id));
            HIP_FATAL(ghip::op_softmax_kqv((const float *)kq, out(sc), out(mk), out(sm), *(const float *)sc->src1->data,
                                           ((const int32_t *)mk->src1->data)[0], tb.exp, sm->ne[0], sm->ne[2], dptr(vv),
                                           vv->nb[1], vv->nb[2], vv->ne[1], (float *)dptr(kqv), (float *)dptr(cb), s));
            for (int i = 0; i < p.n; i++) count_node(p.node[i]);
            count_node(t);
            g_fused[8].fetch_add(1, std::memory_order_relaxed);
            p = Pending{};
            return true;
        }
    }
    // silu -> mul(silu, b): complete
    if (p.n == 1 && last->op == gabi::OP_SILU && t->op == gabi::OP_MUL && same_tensor(t->src0, last) && dev_f32(t) &&
        same_shape(t, last) && dev_f32(t->src1) && same_shape(t, t->src1)) {
        const OpTables &tb = op_tables(id, s);
        // one row (decode): hold it for the q4_0 GEMV that follows (norm_fold)
        NormChain c;
        c.kind = 2;
        c.a = (const float *)dptr(last->src0);
        c.b = (const float *)dptr(t->src1);
        c.norm = (float *)dptr(last);
        c.out = (float *)dptr(t);
        c.table = tb.silu;
        c.ncols = t->ne[0];
        auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
        bool fold = silu_fold_enabled() && !exact_mode() && gabi::nrows(t) == 1 && c.ncols % 64 == 0 &&
                    c.ncols <= 16384 && al(c.a) && al(c.b) && al(c.norm) && al(c.out);
        for (const tensor *o : {(const tensor *)last, (const tensor *)t})
            for (const tensor *i : {(const tensor *)last->src0, (const tensor *)t->src1})
                if (dev_overlap(o, i)) fold = false;
        if (x9_chain_ok(c.ncols, gabi::nrows(t)) && t->ne[2] == 1 && t->ne[3] == 1 && al(c.a) && al(c.b) && al(c.norm) &&
            al(c.out)) {
            fold = true;
            c.nrows = gabi::nrows(t);
        }
        if (fold) {
            c.node[c.nn++] = last;
            c.node[c.nn++] = hold(t);
            c.out_node = c.node[1];
            c.on = true;
            g_norm = c;
            p = Pending{};
            return true;
        }
        HIP_FATAL(hipSetDevice(id));
        HIP_FATAL(ghip::op_silu_mul_f32((const float *)dptr(last->src0), (const float *)dptr(t->src1), (float *)dptr(last),
                                        (float *)dptr(t), t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3], tb.silu, s));
        count_node(last);
        count_node(t);
        g_fused[2].fetch_add(1, std::memory_order_relaxed);
        p = Pending{};
        return true;
    }
    // rope -> cpy(rope, strided device view): complete (the K cache store)
    if (p.n == 1 && last->op == gabi::OP_ROPE && t->op == gabi::OP_CPY && same_tensor(t->src0, last) && t->src1 &&
        t->src1->backend == gabi::BACKEND_GPU && t->src1->extra &&
        (t->src1->type == gabi::TYPE_F16 || t->src1->type == gabi::TYPE_F32) && t->src1->ne[3] == 1 &&
        t->src1->ne[0] * t->src1->ne[1] * t->src1->ne[2] == last->ne[0] * last->ne[1] * last->ne[2] &&
        !overlaps(t->src1, last) && !overlaps(t->src1, last->src0)) {
        p = Pending{};
        run_device_op(last, t);
        count_node(t);
        g_fused[3].fetch_add(1, std::memory_order_relaxed);
        return true;
    }
    // f16 mul_mat -> cpy(permute(mul_mat, 0, 2, 1, 3), contiguous f32): complete (KQV_merged_contiguous)
    if (p.n == 1 && last->op == gabi::OP_MUL_MAT && t->op == gabi::OP_CPY && t->src0 && t->src0->op == gabi::OP_PERMUTE &&
        same_tensor(t->src0->src0, last)) {
        const tensor *m = t->src0, *cb = t->src1;
        if (m->ne[0] == last->ne[0] && m->ne[1] == last->ne[2] && m->ne[2] == last->ne[1] && m->ne[3] == 1 &&
            last->ne[3] == 1 && m->nb[0] == 4 && m->nb[1] == last->nb[2] && m->nb[2] == last->nb[1] && dev_f32(cb) &&
            gabi::nbytes(cb) == gabi::nbytes(last) && !overlaps(cb, last) && !overlaps(cb, last->src0) &&
            !overlaps(cb, last->src1)) {
            p = Pending{};
            run_device_op(last, t);
            count_node(t);
            g_fused[4].fetch_add(1, std::memory_order_relaxed);
            return true;
        }
    }
    // pending silu, then a q4_0 mul_mat that neither reads nor overwrites its buffers: run it now
    if (p.n == 1 && last->op == gabi::OP_SILU && t->op == gabi::OP_MUL_MAT && t->src0 &&
        t->src0->type == gabi::TYPE_Q4_0 && t->backend == gabi::BACKEND_GPU && t->src1 &&
        t->src1->backend == gabi::BACKEND_GPU && !overlaps(t->src1, last) && !overlaps(t, last) &&
        !overlaps(t, last->src0)) {
        count_node(t);
        g_fused[5].fetch_add(1, std::memory_order_relaxed);
        mul_mat_node(t->src0, t->src1, t);
        return true;
    }
    return false;
}

// ---- sibling q4_0 GEMVs.  ggml visits a LLaMA layer depth first, so the mul_mats that share an
// input are not adjacent (wk, rope K, cpy K, wv, cpy V, wq, ...; w1, silu, w3).  A q4_0 mul_mat
// with device operands opens a group; the device-only nodes that follow are held
// behind it ("after" nodes, replayed in arrival order once the group has run), and a later q4_0
// mul_mat with the same src1 joins the group when running it ahead of the held nodes is safe: it
// reads none of their outputs and its output overlaps none of their operands.  The group is one
// multi-matrix GEMV launch (ggml_hip_mul_mat_q4_0_multi), bit-identical to separate launches.
struct Group {
    int n = 0, na = 0;
    tensor *mm[4] = {};
    tensor *after[16] = {};
    NormChain norm;                // the held norm chain the GEMVs run in their prologue (or off)
};
Group g_grp;
void execute_node(tensor *t);

// last byte + 1 of a device tensor's storage, strides included (views, permutes)
size_t span_bytes(const tensor *t) {
    if (gabi::blck_size(t->type) != 1) return gabi::nbytes(t);
    size_t last = gabi::type_size(t->type);
    for (int i = 0; i < 4; i++) last += (size_t)(t->ne[i] - 1) * t->nb[i];
    return last;
}
bool dev_overlap(const tensor *a, const tensor *b) {
    if (!a || !b || a->backend != gabi::BACKEND_GPU || b->backend != gabi::BACKEND_GPU || !a->extra || !b->extra) return false;
    const char *pa = dptr(a), *pb = dptr(b);
    return pa < pb + span_bytes(b) && pb < pa + span_bytes(a);
}

bool main_device_only_split(int64_t M) {
    int active = 0, only = -1;
    for (int id = 0; id < g_device_count; id++) {
        int64_t lo, hi;
        split_range(M, id, &lo, &hi);
        if (lo < hi) active++, only = id;
    }
    return active == 1 && only == g_main_device;
}

bool group_mm_ok(const tensor *t) {
    if (!fuse_enabled() || t->op != gabi::OP_MUL_MAT || !t->src0 || t->src0->type != gabi::TYPE_Q4_0) return false;
    const tensor *a = t->src0, *b = t->src1;
    if (!b || t->backend != gabi::BACKEND_GPU || !t->extra || b->backend != gabi::BACKEND_GPU || !b->extra || !a->extra)
        return false;
    if (!supported_mul_mat(a, b, t) || !is_contiguous(a) || !is_contiguous(b) || !is_contiguous(t)) return false;
    if (b->ne[1] < 1 || b->ne[2] != 1 || b->ne[3] != 1 || a->ne[2] != 1 || a->ne[3] != 1) return false;
    if (a->backend == gabi::BACKEND_GPU) return true;
    return a->backend == gabi::BACKEND_GPU_SPLIT && main_device_only_split(a->ne[1]);
}

bool group_after_ok(const tensor *t) {
    auto dev = [](const tensor *x) { return x && x->backend == gabi::BACKEND_GPU && x->extra; };
    // a CPY node is a view of its target (src1) that llama.cpp does not hand to assign_buffers:
    // its own backend says nothing, the target's does
    if (t->op != gabi::OP_CPY && !dev(t)) return false;
    switch (t->op) {
        case gabi::OP_ADD:
        case gabi::OP_MUL:
            return dev(t->src0) && dev(t->src1);
        case gabi::OP_SILU:
        case gabi::OP_RMS_NORM:
        case gabi::OP_SOFT_MAX:
            return dev(t->src0);
        case gabi::OP_SCALE:
        case gabi::OP_DIAG_MASK_INF:
        case gabi::OP_ROPE:
            return dev(t->src0) && host_scalar_param(t->src1);
        case gabi::OP_CPY:
            return dev(t->src0) && dev(t->src1);
        case gabi::OP_MUL_MAT:
            return t->src0 && t->src0->type == gabi::TYPE_F16 && dev(t->src0) && dev(t->src1);
        default:
            return false;
    }
}

// may q4_0 mul_mat m run before every held node and beside the current members?
bool norm_feeds(const NormChain &c, const tensor *m);
bool group_join_ok(const tensor *m) {
    const Group &g = g_grp;
    if (g.n >= 4 || !same_tensor(m->src1, g.mm[0]->src1) || m->src0->ne[0] != g.mm[0]->src0->ne[0]) return false;
    if (g.norm.on && !norm_feeds(g.norm, m)) return false;
    for (int i = 0; i < g.n; i++)
        if (dev_overlap(m, g.mm[i]) || dev_overlap(m, g.mm[i]->src1)) return false;
    for (int i = 0; i < g.na; i++) {
        const tensor *A = g.after[i];
        if (dev_overlap(m, A) || dev_overlap(m, A->src0) || dev_overlap(m, A->src1)) return false;
        if (dev_overlap(A, m->src1) || dev_overlap(A, m->src0)) return false;
        if (A->op == gabi::OP_CPY && (dev_overlap(A->src1, m->src1) || dev_overlap(A->src1, m->src0))) return false;
    }
    return true;
}

bool trace_nodes() {
    static const bool on = getenv("GGML_HIP_TRACE_NODES") != nullptr;
    return on;
}

// ---- the independent elementwise nodes a group holds (rope K -> K cache, V -> V cache, rope Q):
// one launch for up to four of them when none reads or writes what another writes
struct ElemRW {
    const tensor *r[2];
    const tensor *w[2];
};
bool dev_t(const tensor *x) { return x && x->backend == gabi::BACKEND_GPU && x->extra; }

bool rope_elem(const tensor *t, ghip::ElemOp &op) {
    const tensor *a = t->src0, *b = t->src1;
    if (t->op != gabi::OP_ROPE || !dev_t(a) || !dev_t(t) || a->type != gabi::TYPE_F32 || t->type != gabi::TYPE_F32 ||
        !host_scalar_param(b))
        return false;
    const int n_past = ((const int32_t *)b->data)[0], n_dims = ((const int32_t *)b->data)[1];
    if (((const int32_t *)b->data)[2] != 0 || !same_shape(a, t) || a->nb[0] != 4 || t->nb[0] != 4 || a->ne[0] % 2 ||
        n_dims % 2 || n_past < 0)
        return false;
    const int64_t np = a->ne[0] / 2;
    const float *cs = rope_table(g_main_device, a->ne[0], n_dims, (int64_t)n_past + a->ne[2], g_dev[g_main_device].stream);
    op = ghip::ElemOp{};
    op.kind = 0;
    op.x = dptr(a);
    op.d = dptr(t);
    op.cs = (const float2 *)(cs + (size_t)n_past * np * 2);
    op.npairs = (int)np;
    op.n = np * a->ne[1] * a->ne[2] * a->ne[3];
    op.ne0 = a->ne[0], op.ne1 = a->ne[1], op.ne2 = a->ne[2];
    op.nbx1 = a->nb[1], op.nbx2 = a->nb[2], op.nbx3 = a->nb[3];
    op.nbd1 = t->nb[1], op.nbd2 = t->nb[2], op.nbd3 = t->nb[3];
    return true;
}
bool cpy_target_ok(const tensor *t) {     // a CPY node F32 -> F32/F16 between device tensors, 3-d
    const tensor *a = t->src0, *b = t->src1;
    return t->op == gabi::OP_CPY && dev_t(a) && dev_t(b) && a->type == gabi::TYPE_F32 &&
           (b->type == gabi::TYPE_F32 || b->type == gabi::TYPE_F16) && a->ne[3] == 1 && b->ne[3] == 1 &&
           a->ne[0] * a->ne[1] * a->ne[2] == b->ne[0] * b->ne[1] * b->ne[2];
}
void set_copy_target(ghip::ElemOp &op, const tensor *b) {
    op.c = dptr(b);
    op.f16 = b->type == gabi::TYPE_F16;
    op.ne10 = b->ne[0], op.ne11 = b->ne[1], op.nb10 = b->nb[0], op.nb11 = b->nb[1], op.nb12 = b->nb[2];
}

// batches a prefix of the held list; returns how many held nodes it ran
int run_elem_prefix(tensor *const *held, int nh) {
    if (!fuse_enabled()) return 0;
    ghip::ElemBatch b{};
    ElemRW rw[ghip::ELEM_MAX];
    int used = 0;
    while (b.nops < ghip::ELEM_MAX && used < nh) {
        tensor *t = held[used];
        ghip::ElemOp op;
        ElemRW e{{nullptr, nullptr}, {nullptr, nullptr}};
        int take = 0;
        if (rope_elem(t, op)) {
            e.r[0] = t->src0;
            e.w[0] = t;
            take = 1;
            if (used + 1 < nh && held[used + 1]->src0 == t && cpy_target_ok(held[used + 1]) &&
                t->ne[3] == 1 && !dev_overlap(held[used + 1]->src1, t) && !dev_overlap(held[used + 1]->src1, t->src0)) {
                set_copy_target(op, held[used + 1]->src1);
                e.w[1] = held[used + 1]->src1;
                take = 2;
            }
        } else if (cpy_target_ok(t)) {
            const tensor *a = t->src0;
            op = ghip::ElemOp{};
            op.kind = 1;
            op.x = dptr(a);
            op.n = a->ne[0] * a->ne[1] * a->ne[2];
            op.ne0 = a->ne[0], op.ne1 = a->ne[1];
            op.nbx1 = a->nb[0], op.nbx2 = a->nb[1], op.nbx3 = a->nb[2];
            set_copy_target(op, t->src1);
            e.r[0] = a;
            e.w[0] = t->src1;
            take = 1;
        } else {
            break;
        }
        // independent of every entry already in the batch (they run concurrently)
        bool ok = true;
        for (int q = 0; q < b.nops && ok; q++)
            for (const tensor *w : rw[q].w)
                for (const tensor *x : {e.r[0], e.r[1], e.w[0], e.w[1]})
                    if (w && x && dev_overlap(w, x)) ok = false;
        for (int q = 0; q < b.nops && ok; q++)
            for (const tensor *w : e.w)
                for (const tensor *x : rw[q].r)
                    if (w && x && dev_overlap(w, x)) ok = false;
        if (!ok) break;
        rw[b.nops] = e;
        b.op[b.nops++] = op;
        used += take;
    }
    if (b.nops < 2) return 0;
    HIP_FATAL(hipSetDevice(g_main_device));
    HIP_FATAL(ghip::op_elem_batch(b, g_dev[g_main_device].stream));
    for (int i = 0; i < used; i++) count_node(held[i]);
    g_fused[7].fetch_add(1, std::memory_order_relaxed);
    return used;
}

void launch_norm_chain(const NormChain &c) {
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    if (c.kind == 2)
        HIP_FATAL(ghip::op_silu_mul_f32(c.a, c.b, c.norm, c.out, c.ncols * c.nrows, c.table, g_dev[id].stream));
    else
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32(c.a, c.b, c.sum, c.norm, c.w, c.out, c.ncols, c.nrows, g_dev[id].stream));
    for (int i = 0; i < c.nn; i++) count_node(c.node[i]);
    g_fused[c.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
}
void flush_norm() {
    const NormChain c = g_norm;
    g_norm = NormChain{};
    if (c.on) launch_norm_chain(c);
}
// may a held norm chain's output feed q4_0 mul_mat m through its GEMV prologue?
bool norm_feeds(const NormChain &c, const tensor *m) {
    if (!c.on || !same_tensor(m->src1, c.out_node) || m->src1->ne[1] != c.nrows || m->src0->ne[0] != c.ncols) return false;
    // m's output must not alias anything the prologue reads or workgroup 0 stores
    const char *y = dptr(m);
    const size_t yb = span_bytes(m), row = (size_t)c.ncols * (size_t)c.nrows * 4;
    for (const void *q : {(const void *)c.a, (const void *)c.b, (const void *)c.w, (const void *)c.sum,
                          (const void *)c.norm, (const void *)c.out})
        if (q && (const char *)q < y + yb && y < (const char *)q + row) return false;
    return true;
}

// prefill (N > IMG_MIN_N) mul_mats of resident weights take k_gemm9 on an fp6 image built once
// (mul_mat_node's rule, here for a group's members)
void ensure_group_images(const Group &g) {
    const int64_t N = g.mm[0]->src1->ne[1];
    if (N <= IMG_MIN_N || exact_mode() || (gemm_version() != 8 && gemm_version() != 10)) return;
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    for (int i = 0; i < g.n; i++) wimage_ensure(id, dptr(g.mm[i]->src0), g.mm[i]->src0->ne[0], g.mm[i]->src0->ne[1], g_dev[id].stream);
}

// A held prefill chain and the q4_0 mul_mats that consume it: when every member takes k_gemm9 on an
// fp6 image, the chain's launch writes the x image beside its f32 output and the members run as one
// k_gemm9 launch on it (no k_prep9_x; the image is bitwise gemm9_prep_x's of the chain's output, so y
// is bitwise the unfused path's).  false: not every member qualifies (nothing launched).
bool flush_group_x9(const Group &g) {
    const NormChain &c = g.norm;
    const int id = g_main_device;
    const int64_t K = c.ncols, N = c.nrows;
    if (exact_mode() || gemm_version() != 10 || N * K >= ((int64_t)1 << 31)) return false;
    const void *img[4];
    int64_t M[4], ldy[4];
    float *y[4];
    for (int i = 0; i < g.n; i++) {
        const tensor *a = g.mm[i]->src0;
        int fmt = 0;
        M[i] = ldy[i] = a->ne[1];
        img[i] = wimage_find(id, dptr(a), K, M[i], &fmt);
        if (!img[i] || fmt != 9 || M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31) || M[i] >= (1 << 30)) return false;
        y[i] = (float *)dptr(g.mm[i]);
    }
    hipStream_t s = g_dev[id].stream;
    void *ws = nullptr;
    if (stream_workspace(id, s, workspace_bytes_mm(K, N, 0), &ws) != GGML_HIP_OK) return false;
    void *xws = (char *)ws + ws_g8x_offset(K, N);
    const int64_t Np = ghip::gemm9_np(N);
    HIP_FATAL(hipSetDevice(id));
    if (c.kind == 2)
        HIP_FATAL(ghip::op_silu_mul_f32_x9(c.a, c.b, c.norm, c.out, K, N, c.table, xws, Np, s));
    else
        HIP_FATAL(ghip::op_add_rms_norm_mul_f32_x9(c.a, c.b, c.sum, c.norm, c.w, c.out, K, N, xws, Np, s));
    HIP_FATAL(ghip::gemm9_run_multi(g.n, img, M, K, xws, N, y, ldy, s));
    for (int i = 0; i < c.nn; i++) count_node(c.node[i]);
    for (int i = 0; i < g.n; i++) count_node(g.mm[i]);
    g_fused[c.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
    g_fused[11].fetch_add(1, std::memory_order_relaxed);
    if (g.n > 1) g_fused[6].fetch_add(1, std::memory_order_relaxed);
    return true;
}

void flush_group() {
    const Group g = g_grp;
    g_grp = Group{};
    if (g.n > 0) ensure_group_images(g);
    if (g.norm.on && g.norm.nrows > 1) {  // a held prefill chain: the x image fold, or its own launch first
        const bool done = flush_group_x9(g);
        if (!done) launch_norm_chain(g.norm);
        if (done) {
            const int k = run_elem_prefix(g.after, g.na);
            for (int i = k; i < g.na; i++) execute_node(g.after[i]);
            return;
        }
    } else if (g.norm.on) {               // the GEMVs run the held norm chain in their prologue
        const void *w[4];
        int64_t m[4], ldy[4];
        float *y[4];
        for (int i = 0; i < g.n; i++) {
            w[i] = dptr(g.mm[i]->src0);
            m[i] = ldy[i] = g.mm[i]->src0->ne[1];
            y[i] = (float *)dptr(g.mm[i]);
        }
        const ghip::GemvNorm nrm{g.norm.a, g.norm.w, g.norm.sum, g.norm.norm, g.norm.out, g.norm.kind, g.norm.table};
        HIP_FATAL(hipSetDevice(g_main_device));
        HIP_FATAL(ghip::gemv_q4_0_multi_norm(g.n, w, m, g.norm.ncols, g.norm.b, nrm, y, ldy,
                                             g_dev[g_main_device].info, g_dev[g_main_device].stream));
        for (int i = 0; i < g.norm.nn; i++) count_node(g.norm.node[i]);
        for (int i = 0; i < g.n; i++) count_node(g.mm[i]);
        g_fused[g.norm.kind == 2 ? 2 : 0].fetch_add(1, std::memory_order_relaxed);
        g_fused[g.norm.kind == 2 ? 10 : 9].fetch_add(1, std::memory_order_relaxed);
        if (g.n > 1) g_fused[6].fetch_add(1, std::memory_order_relaxed);
        const int done = run_elem_prefix(g.after, g.na);
        for (int i = done; i < g.na; i++) execute_node(g.after[i]);
        return;
    }
    if (trace_nodes()) fprintf(stderr, "group flush: %d mul_mats (%s ...), %d held nodes\n", g.n, g.mm[0]->name, g.na);
    if (g.n == 1) {
        count_node(g.mm[0]);
        mul_mat_node(g.mm[0]->src0, g.mm[0]->src1, g.mm[0]);
    } else if (g.n > 1) {
        const void *w[4];
        int64_t m[4];
        float *y[4];
        for (int i = 0; i < g.n; i++) {
            w[i] = dptr(g.mm[i]->src0);
            m[i] = g.mm[i]->src0->ne[1];
            y[i] = (float *)dptr(g.mm[i]);
            count_node(g.mm[i]);
        }
        HIP_FATAL(hipSetDevice(g_main_device));
        const int rc = ggml_hip_mul_mat_q4_0_multi(g.n, w, m, g.mm[0]->src0->ne[0], (const float *)dptr(g.mm[0]->src1),
                                                   g.mm[0]->src1->ne[1], y, g_dev[g_main_device].stream);
        if (rc != GGML_HIP_OK) op_abort(g.mm[0], "sibling q4_0 GEMV group failed");
        g_fused[6].fetch_add(1, std::memory_order_relaxed);
    }
    const int done = run_elem_prefix(g.after, g.na);
    for (int i = done; i < g.na; i++) execute_node(g.after[i]);   // the ordinary path, fusion included
}

// runs (or defers) one taken node; the ith == 0 COMPUTE phase of ggml_hip_compute_forward
void execute_node(tensor *t) {
    const int op = t->op;
    if (op == gabi::OP_RESHAPE || op == gabi::OP_VIEW || op == gabi::OP_PERMUTE || op == gabi::OP_TRANSPOSE) {
        count_node(t);                      // no data touched: a pending chain stays pending
        return;
    }
    // a held norm chain: a GEMV that consumes it opens a group that runs it in its prologue
    auto open_norm_group = [&]() {
        if (!g_norm.on || g_grp.n != 0 || g_pend.n != 0 || !group_mm_ok(t) || !norm_feeds(g_norm, t)) return false;
        g_grp.mm[0] = hold(t);
        g_grp.n = 1;
        g_grp.norm = g_norm;
        g_norm = NormChain{};
        return true;
    };
    if (g_norm.on) {
        if (open_norm_group()) return;
        flush_norm();                         // anything else: the chain runs as its own launch
    }
    if (g_grp.n > 0) {
        if (group_mm_ok(t) && group_join_ok(t)) {
            g_grp.mm[g_grp.n++] = hold(t);
            return;
        }
        if (trace_nodes())
            fprintf(stderr, "group: %s not joined (mm_ok %d, join_ok %d, after_ok %d)\n", t->name, (int)group_mm_ok(t),
                    group_mm_ok(t) ? (int)group_join_ok(t) : -1, (int)group_after_ok(t));
        if (!(op == gabi::OP_MUL_MAT && t->src0 && t->src0->type != gabi::TYPE_F16) && group_after_ok(t) &&
            g_grp.na < 16) {
            g_grp.after[g_grp.na++] = hold(t);
            return;
        }
        flush_group();                        // its held nodes may complete a norm chain t consumes
        if (open_norm_group()) return;
        if (g_norm.on) flush_norm();
    }
    if (g_pend.n == 0 && group_mm_ok(t)) {
        g_grp.mm[0] = hold(t);
        g_grp.n = 1;
        return;
    }
    if (g_pend.n > 0) {
        if (try_fuse(t)) return;
        flush_pending();
        if (group_mm_ok(t)) {
            g_grp.mm[0] = hold(t);
            g_grp.n = 1;
            return;
        }
    }
    if (deferrable(t)) {
        g_pend.node[g_pend.n++] = hold(t);
        return;
    }
    if (t->op == gabi::OP_MUL_MAT && t->src0 && t->src0->type != gabi::TYPE_F16) {
        count_node(t);
        ggml_hip_mul_mat((const ggml_tensor *)t->src0, (const ggml_tensor *)t->src1, (ggml_tensor *)t);
    } else {
        run_device_op(t);
    }
}

}  // namespace

// every backend entry point that can touch device memory outside the node sequence
// launch recording on the hook path: opt-in (GGML_HIP_GRAPH=1 or ggml_hip_debug_set_graph(1)).  It cuts
// the host walk of a LLaMA-7B decode eval from 1.36 to 0.59 ms, but the eval is device bound (~330
// kernels, ~2.3 us per boundary) and HIP's graph replay leaves a ~100 us gap every 16 nodes: equal or
// 2-3 % slower end to end, so eager launches stay the default.
static std::atomic<int> &graph_flag() {
    static std::atomic<int> f([] {
        const char *e = getenv("GGML_HIP_GRAPH");
        return e ? atoi(e) : 0;
    }());
    return f;
}
static inline bool graph_enabled() { return graph_flag().load(std::memory_order_relaxed) != 0; }
static inline void graph_apply_mode() {          // 1: HIP graphs, 2: launcher thread (launch.h)
    static int applied = -1;
    const int m = graph_flag().load(std::memory_order_relaxed);
    if (m != applied && m != 0) ghip::rec_set_mode(m);
    applied = m;
}

static inline void flush_deferred() {
    if (g_grp.n > 0) flush_group();
    if (g_norm.on) flush_norm();
    if (g_pend.n > 0) flush_pending();
    ghip::rec_flush_at("entry point");        // and submit the recorded launches (launch.h)
}

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

void ggml_init_hip(void) { ensure_init(); }

void ggml_hip_set_tensor_split(const float *tensor_split) {
    // ggml-cuda.cu:1863-1882
    ensure_init();
    if (!tensor_split) return;
    bool all_zero = true;
    for (int i = 0; i < g_device_count; i++)
        if (tensor_split[i] != 0.0f) all_zero = false;
    if (all_zero) return;
    split_fractions(tensor_split, g_device_count, g_tensor_split);
}

bool ggml_hip_can_mul_mat(const struct ggml_tensor *src0_, const struct ggml_tensor *src1_, struct ggml_tensor *dst_) {
    // ggml-cuda.cu:2595-2610, restricted to the q4_0 path this backend implements
    const tensor *src0 = (const tensor *)src0_, *src1 = (const tensor *)src1_, *dst = (const tensor *)dst_;
    if (!supported_mul_mat(src0, src1, dst)) return false;
    // no device: decline, so ggml.c plans and runs its own CPU mul_mat (the reference would route
    // the op here regardless and fail inside ggml_cuda_mul_mat)
    ensure_init();
    if (g_device_count == 0) return false;
    if (dst->ne[0] >= 32 && dst->ne[1] >= 32 && src1->ne[0] >= 32) return true;
    // Decode (N < 32) of a host-resident Q4_0 weight: the reference declines it (each call would
    // re-upload the weight, ggml-cuda.cu:2496-2502), so the arch/ frontends, which never offload,
    // decode on the CPU.  Here the weight-residency cache keeps the weight on the device after its
    // first use, so a weight of at least GGML_HIP_DECODE_MIN_WEIGHTS elements (default 2^19: one
    // LLaMA/Falcon projection is 2^24) is taken at any N; smaller ones stay on ggml's CPU op.
    return src0->type == gabi::TYPE_Q4_0 && wcache_enabled() &&
           (uint64_t)src0->ne[0] * (uint64_t)src0->ne[1] >= (uint64_t)decode_min_weights();
}

size_t ggml_hip_mul_mat_get_wsize(const struct ggml_tensor *, const struct ggml_tensor *, struct ggml_tensor *) {
    return 0;
}

void ggml_hip_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst) {
    ensure_init();
    flush_deferred();
    mul_mat_node((const tensor *)src0, (const tensor *)src1, (tensor *)dst);
}

}  // extern "C"

namespace {
// the q4_0 mul_mat of one node; leaves a pending fusion chain alone (try_fuse checked that the two
// touch disjoint buffers)
void mul_mat_node(const tensor *src0, const tensor *src1, tensor *dst) {
    // ggml_cuda_mul_mat -> ggml_cuda_op (ggml-cuda.cu:2671-2690, 2286-2567)
    if (!supported_mul_mat(src0, src1, dst)) {
        fprintf(stderr, "ggml_hip_mul_mat: unsupported operands (need contiguous Q4_0 x F32 -> F32, K %% 64 == 0)\n");
        abort();
    }
    const int64_t K = src0->ne[0], M = src0->ne[1], N = src1->ne[1];
    const int64_t nbatch = src0->ne[2] * src0->ne[3];
    // a row split that puts every row on the main device (one device, or a tensor_split that gives
    // the others nothing) is an ordinary device matrix: direct output, no gather, no synchronize
    // (llama.cpp marks every layer matrix GPU_SPLIT, llama.cpp:1059-1076)
    bool split = src0->backend == gabi::BACKEND_GPU_SPLIT;
    if (split) {
        int active = 0, only = -1;
        for (int id = 0; id < g_device_count; id++) {
            int64_t lo, hi;
            split_range(M, id, &lo, &hi);
            if (lo < hi) active++, only = id;
        }
        if (active == 1 && only == g_main_device) split = false;
    }
    const bool src0_dev = on_device(src0);
    const bool src1_dev = src1->backend == gabi::BACKEND_GPU;
    const bool dst_dev = dst->backend == gabi::BACKEND_GPU;
    const size_t wrow = (size_t)(K / QK) * Q4B;
    const int saved = current_device();
    const int main_id = g_main_device;
    uint64_t call_id;
    {
        std::lock_guard<std::mutex> lk(g_wc_mu);
        call_id = ++g_wc_clock;
    }
    // Row split over devices (ggml_cuda_op, ggml-cuda.cu:2286-2567): every device's slice is
    // enqueued before anything waits, so the devices run concurrently; the host synchronizes each
    // device once at the end (the reference: main-device sync first, per-device sync last,
    // 2348-2351 / 2546-2552).  Other devices start after the main stream's work that produced
    // src1 (event); a non-main slice [N][rows] comes back with ONE contiguous peer copy into a
    // main-device staging buffer and ONE 2-D copy into dst on the main stream (which waits for it).
    if (split) {
        HIP_FATAL(hipSetDevice(main_id));
        HIP_FATAL(GHIP_SYNC(hipEventRecord)(g_dev[main_id].ev_a, g_dev[main_id].stream));
    }
    std::vector<std::vector<std::pair<void *, size_t>>> tmps(g_device_count);
    std::vector<bool> used(g_device_count, false);
    bool need_sync = !dst_dev || split || !src0_dev;   // host dst, gathers, host weights (cache)
    for (int id = 0; id < g_device_count; id++) {
        if (!split && id != main_id) continue;
        int64_t lo = 0, hi = M;
        if (split) split_range(M, id, &lo, &hi);
        if (lo == hi) continue;
        used[id] = true;
        const int64_t rows = hi - lo;
        HIP_FATAL(hipSetDevice(id));
        hipStream_t s = g_dev[id].stream;
        auto tmp_alloc = [&](int dev, size_t bytes) {
            size_t a = 0;
            void *p = pool_malloc(dev, bytes, &a);
            tmps[dev].push_back({p, a});
            return p;
        };
        if (split && id != main_id) HIP_FATAL(GHIP_SYNC(hipStreamWaitEvent)(s, g_dev[main_id].ev_a, 0));
        for (int64_t b = 0; b < nbatch; b++) {
            // weights: resident slice, or upload the row slice (the reference re-uploads every
            // call too, ggml-cuda.cu:2496-2502)
            const void *w;
            bool w_resident = true;                // device weight or cached copy: may get an int8 image
            if (src0_dev) {
                const auto *ex = (const ggml_tensor_extra_gpu *)src0->extra;
                w = (const char *)ex->data_device[id] + (size_t)b * rows * wrow;
            } else if (wcache_enabled()) {
                w = wcache_get(id, (const char *)src0->data + (size_t)b * src0->nb[2] + lo * wrow, rows * wrow, s,
                               call_id);
            } else {
                void *p = tmp_alloc(id, rows * wrow);
                HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(p, (const char *)src0->data + (size_t)b * src0->nb[2] + lo * wrow, rows * wrow,
                                         hipMemcpyHostToDevice, s));
                w = p;
                w_resident = false;
            }
            // prefill (N > IMG_MIN_N) of a resident weight: build its image once (fp6 for k_gemm9, int8
            // under version 8; a failure to allocate it leaves the q4_0 bytes to k_gemm7 / split-K)
            if (w_resident && N > IMG_MIN_N && !exact_mode() && (gemm_version() == 8 || gemm_version() == 10) &&
                (src0_dev || wcache_images_enabled())) {
                const bool had = wimage_find(id, w, K, rows) != nullptr;
                if (wimage_ensure(id, w, K, rows, s) && !had && !src0_dev)
                    wcache_note_image(id, w, image_format() == 9 ? ghip::gemm9_w_bytes(K, rows) : ghip::gemm8_w_bytes(K, rows));
            }
            // activations
            const float *x;
            const size_t xbytes = (size_t)N * K * 4;
            if (src1_dev && id == main_id) {
                x = (const float *)((const char *)((const ggml_tensor_extra_gpu *)src1->extra)->data_device[id] +
                                    (size_t)b * src1->nb[2]);
            } else if (src1_dev) {
                void *p = tmp_alloc(id, xbytes);
                const char *srcp = (const char *)((const ggml_tensor_extra_gpu *)src1->extra)->data_device[main_id] +
                                   (size_t)b * src1->nb[2];
                HIP_FATAL(GHIP_SYNC(hipMemcpyPeerAsync)(p, id, srcp, main_id, xbytes, s));
                x = (const float *)p;
            } else {
                void *p = tmp_alloc(id, xbytes);
                HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(p, (const char *)src1->data + (size_t)b * src1->nb[2], xbytes,
                                         hipMemcpyHostToDevice, s));
                x = (const float *)p;
            }
            // output
            float *y;
            int64_t ldy;
            const bool direct = dst_dev && !split && id == main_id;
            if (direct) {
                y = (float *)((char *)((ggml_tensor_extra_gpu *)dst->extra)->data_device[id] + (size_t)b * dst->nb[2]);
                ldy = M;
            } else {
                y = (float *)tmp_alloc(id, (size_t)N * rows * 4);
                ldy = rows;
            }
            if (mul_mat_dev(w, K, rows, x, N, y, ldy, 0, s) != GGML_HIP_OK) {
                fprintf(stderr, "ggml_hip_mul_mat: %s\n", g_last_error.c_str());
                abort();
            }
            if (direct) continue;
            // y slice [N][rows] -> dst[n*M + lo + i]
            if (!dst_dev) {
                char *dbase = (char *)dst->data + (size_t)b * dst->nb[2] + lo * 4;
                HIP_FATAL(GHIP_SYNC(hipMemcpy2DAsync)(dbase, M * 4, y, rows * 4, rows * 4, N, hipMemcpyDeviceToHost, s));
                continue;
            }
            char *dbase = (char *)((ggml_tensor_extra_gpu *)dst->extra)->data_device[main_id] + (size_t)b * dst->nb[2] +
                          lo * 4;
            if (id == main_id) {
                HIP_FATAL(GHIP_SYNC(hipMemcpy2DAsync)(dbase, M * 4, y, rows * 4, rows * 4, N, hipMemcpyDeviceToDevice, s));
                continue;
            }
            void *stage = tmp_alloc(main_id, (size_t)N * rows * 4);
            HIP_FATAL(GHIP_SYNC(hipMemcpyPeerAsync)(stage, main_id, y, id, (size_t)N * rows * 4, s));
            HIP_FATAL(GHIP_SYNC(hipEventRecord)(g_dev[id].ev_b, s));
            HIP_FATAL(hipSetDevice(main_id));
            HIP_FATAL(GHIP_SYNC(hipStreamWaitEvent)(g_dev[main_id].stream, g_dev[id].ev_b, 0));
            HIP_FATAL(GHIP_SYNC(hipMemcpy2DAsync)(dbase, M * 4, stage, rows * 4, rows * 4, N, hipMemcpyDeviceToDevice,
                                       g_dev[main_id].stream));
            HIP_FATAL(hipSetDevice(id));
        }
    }
    // temporaries are reusable after this (ggml-cuda.cu:2546-2566); a call whose operands were all
    // device resident stays stream-ordered (full offload: the next op runs on the same stream)
    for (int id = 0; id < g_device_count; id++) {
        const bool main_staged = id == main_id && !tmps[id].empty();
        if (!used[id] && !main_staged) continue;
        if (need_sync || !tmps[id].empty()) {
            HIP_FATAL(hipSetDevice(id));
            HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(g_dev[id].stream));
        }
        for (auto &t : tmps[id]) pool_free(id, t.first, t.second);
    }
    HIP_FATAL(hipSetDevice(saved));
}
}  // namespace

extern "C" {

void ggml_hip_mul(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst) {
    // ggml_cuda_mul (ggml-cuda.cu:2580-2583): the MUL node on the device, whatever dst->op says
    ensure_init();
    flush_deferred();
    tensor node = *(const tensor *)dst;
    node.op = gabi::OP_MUL;
    node.src0 = (tensor *)src0;
    node.src1 = (tensor *)src1;
    run_device_op(&node);
}

void *ggml_hip_host_malloc(size_t size) {
    // ggml-cuda.cu:1884-1899
    ensure_init();
    if (getenv("GGML_HIP_NO_PINNED") != nullptr) return nullptr;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, size, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        fprintf(stderr, "WARNING: failed to allocate %.2f MB of pinned memory: %s\n", size / 1024.0 / 1024.0,
                hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

void ggml_hip_host_free(void *ptr) {
    if (ptr) HIP_FATAL(hipHostFree(ptr));
}

void ggml_hip_transform_tensor(void *data, struct ggml_tensor *tensor_) {
    // ggml-cuda.cu:2766-2809
    ensure_init();
    flush_deferred();
    tensor *t = (tensor *)tensor_;
    if ((t->type != gabi::TYPE_Q4_0 && t->type != gabi::TYPE_F32 && t->type != gabi::TYPE_F16) || g_device_count == 0) {
        // A type no device op reads: ggml.c computes the ops that read it on the CPU and asserts
        // CPU operands there (ggml.c:15650), so the tensor stays a CPU tensor, on a host copy this
        // backend owns (the loader may free `data` after the call, llama.cpp:680-683).
        const size_t bytes = gabi::nbytes(t);
        void *h = malloc(bytes ? bytes : 1);
        if (!h) {
            fprintf(stderr, "ggml_hip_transform_tensor: host copy of %zu bytes failed\n", bytes);
            abort();
        }
        memcpy(h, data, bytes);
        {
            std::lock_guard<std::mutex> lk(g_host_copy_mu);
            g_host_copies[t] = h;
        }
        t->data = h;
        t->backend = gabi::BACKEND_CPU;
        t->extra = nullptr;
        return;
    }
    if (t->type != gabi::TYPE_Q4_0 && t->backend == gabi::BACKEND_GPU_SPLIT)
        t->backend = gabi::BACKEND_GPU;   // only the Q4_0 mul_mat reads row-split operands
    const int64_t nrows = gabi::nrows(t);
    const size_t nb1 = t->nb[1];
    auto *extra = new ggml_tensor_extra_gpu;
    memset(extra, 0, sizeof(*extra));
    const int saved = current_device();
    for (int id = 0; id < g_device_count; id++) {
        if (t->backend == gabi::BACKEND_GPU && id != g_main_device) continue;
        int64_t lo, hi;
        if (t->backend == gabi::BACKEND_GPU) {
            lo = 0;
            hi = nrows;
        } else if (t->backend == gabi::BACKEND_GPU_SPLIT) {
            split_range(nrows, id, &lo, &hi);
        } else {
            fprintf(stderr, "ggml_hip_transform_tensor: tensor backend is not GPU\n");
            abort();
        }
        if (lo == hi) continue;
        const size_t size = (size_t)(hi - lo) * nb1;
        HIP_FATAL(hipSetDevice(id));
        void *buf = nullptr;
        HIP_FATAL(hipMalloc(&buf, size));
        HIP_FATAL(GHIP_SYNC(hipMemcpy)(buf, (const char *)data + lo * nb1, size, hipMemcpyHostToDevice));
        extra->data_device[id] = buf;
        own_device_buffer(buf);
    }
    HIP_FATAL(hipSetDevice(saved));
    t->extra = extra;
}

void ggml_hip_free_data(struct ggml_tensor *tensor_) {
    // ggml-cuda.cu:2811-2828
    flush_deferred();
    tensor *t = (tensor *)tensor_;
    {
        std::lock_guard<std::mutex> lk(g_host_copy_mu);
        auto it = g_host_copies.find(t);
        if (it != g_host_copies.end()) {      // a tensor transform_tensor kept on the CPU
            if (t->data == it->second) t->data = nullptr;
            free(it->second);
            g_host_copies.erase(it);
            return;
        }
    }
    if (!on_device(t) || !t->extra) return;
    ensure_init();
    auto *extra = (ggml_tensor_extra_gpu *)t->extra;
    const int saved = current_device();
    for (int id = 0; id < g_device_count; id++) {
        if (!extra->data_device[id] || !release_device_buffer(extra->data_device[id])) continue;
        HIP_FATAL(hipSetDevice(id));
        // int8 prefill images of this weight (any batch slice; the whole tensor's bytes bound them)
        wimage_drop(extra->data_device[id], (size_t)t->nb[3] * (size_t)t->ne[3]);
        HIP_FATAL(GHIP_SYNC(hipFree)(extra->data_device[id]));
    }
    HIP_FATAL(hipSetDevice(saved));
    forget_graph_extra(t, extra);
    t->extra = nullptr;
}

// Graph-tensor offload (ggml-cuda.cu:2830-2904): the tensor becomes a device tensor; its storage
// is its source's (in-place ops and views, at the view's byte offset), its copy target's (CPY), a
// slot of the VRAM scratch ring (scratch: wraps to the start when full, as the reference does),
// or its own zeroed buffer (no_scratch: the KV cache).  Every op of such a graph runs on the
// device (ggml_hip_compute_forward), so activations stay resident across the layer.
// (a pending fused chain reads its tensors' extras when it runs: flush before they are reassigned)
// The first assignment after a graph was computed starts the next eval's graph: its scratch slots
// start at offset 0 again (the previous eval's activations are dead once its outputs were read), so
// every decode eval places its nodes at the same device addresses.  The reference keeps advancing the
// ring across evals; any start is equivalent, and a fixed one lets the launch recorder (launch.h)
// replay the previous eval's graph with only the position-dependent nodes updated.
static void begin_build() {
    if (g_eval_computed) {
        g_eval_computed = false;
        g_scratch_offset = 0;
    }
}
void ggml_hip_assign_buffers(struct ggml_tensor *t) {
    flush_deferred();
    begin_build();
    assign_buffers_impl((tensor *)t, true, false);
}
void ggml_hip_assign_buffers_no_scratch(struct ggml_tensor *t) {
    flush_deferred();
    begin_build();
    assign_buffers_impl((tensor *)t, false, false);
}
void ggml_hip_assign_buffers_force_inplace(struct ggml_tensor *t) {
    flush_deferred();
    begin_build();
    assign_buffers_impl((tensor *)t, false, true);
}

void ggml_hip_set_main_device(int main_device) {
    // ggml-cuda.cu:2906-2918
    ensure_init();
    if (main_device >= g_device_count) {
        fprintf(stderr, "warning: cannot set main_device=%d because there are only %d devices. Using device %d instead.\n",
                main_device, g_device_count, g_device_count - 1);
        main_device = g_device_count - 1;
    }
    if (main_device < 0) main_device = 0;
    g_main_device = main_device;
}

void ggml_hip_set_scratch_size(size_t scratch_size) { g_scratch_size = scratch_size; }

void ggml_hip_free_scratch(void) {
    flush_deferred();
    if (g_scratch) {
        HIP_FATAL(GHIP_SYNC(hipFree)(g_scratch));
        g_scratch = nullptr;
    }
    g_scratch_offset = 0;
}

bool ggml_hip_compute_forward(struct ggml_compute_params *params_, struct ggml_tensor *tensor_) {
    // ggml-cuda.cu:2933-3021: a node is taken when any operand is device resident (MUL_MAT also when
    // can_mul_mat holds for host operands); only ith == 0 in COMPUTE executes (the other threads
    // spin in ggml.c:17285-17287).  Q4_0 mul_mat -> the q4_0 kernels; F16 mul_mat (attention on the
    // KV cache) and the other ops of a LLaMA layer -> ggml_ops.hip; views are free.
    const gabi::compute_params *params = (const gabi::compute_params *)params_;
    tensor *t = (tensor *)tensor_;
    // a host write into cached weights (LoRA apply) invalidates their device copies; INIT runs once per
    // node, before any thread writes (ggml.c:17112-17116)
    if (params->type == gabi::TASK_INIT && t->backend == gabi::BACKEND_CPU && t->data && t->op != gabi::OP_NONE &&
        t->op != gabi::OP_VIEW && t->op != gabi::OP_RESHAPE && t->op != gabi::OP_PERMUTE && t->op != gabi::OP_TRANSPOSE)
        wcache_note_host_write(t->data, span_bytes(t));   // (views of a weight write nothing)
    const bool any_on_device = t->backend == gabi::BACKEND_GPU || on_device(t->src0) ||
                               (t->src1 && t->src1->backend == gabi::BACKEND_GPU);
    bool f16_mul_mat = false;
    switch (t->op) {
        case gabi::OP_MUL_MAT:
            if (t->src0 && t->src0->type == gabi::TYPE_F16) {
                if (!any_on_device) return false;
                f16_mul_mat = true;
                break;
            }
            if (!supported_mul_mat(t->src0, t->src1, t)) return false;
            ensure_init();
            if (g_device_count == 0) return false;
            if (!any_on_device && !ggml_hip_can_mul_mat((const ggml_tensor *)t->src0, (const ggml_tensor *)t->src1,
                                                        (ggml_tensor *)t))
                return false;
            break;
        case gabi::OP_ADD:
        case gabi::OP_MUL:
        case gabi::OP_SILU:
        case gabi::OP_RMS_NORM:
        case gabi::OP_SCALE:
        case gabi::OP_CPY:
        case gabi::OP_DIAG_MASK_INF:
        case gabi::OP_SOFT_MAX:
        case gabi::OP_ROPE:
        case gabi::OP_RESHAPE:
        case gabi::OP_VIEW:
        case gabi::OP_PERMUTE:
        case gabi::OP_TRANSPOSE:
            if (!any_on_device) return false;
            break;
        default:
            return false;
    }
    if (params->ith != 0) return true;
    if (params->type == gabi::TASK_INIT || params->type == gabi::TASK_FINALIZE) return true;
    ensure_init();
    static const bool trace = getenv("GGML_HIP_TRACE_NODES") != nullptr;
    if (trace)
        fprintf(stderr, "node op=%d %-24s src0=%-24s src1=%s\n", t->op, t->name, t->src0 ? t->src0->name : "-",
                t->src1 ? t->src1->name : "-");
    const auto t0 = std::chrono::steady_clock::now();
    (void)f16_mul_mat;
    if (g_grp.n == 0 && g_pend.n == 0 && !g_norm.on) {
        snap_reset();                      // nothing held: the copies are garbage
    } else if (g_snaps.memo.count(t)) {
        flush_deferred();                  // t arrives again: a new graph at the old addresses
    }
    // with the recorder on, the node's launches on the main stream are recorded and submitted as HIP
    // graphs (launch.h)
    g_eval_computed = true;
    const bool use_graph = graph_enabled();
    if (use_graph) graph_apply_mode();
    if (use_graph) ghip::rec_enable(g_dev[g_main_device].stream, true);
    execute_node(t);
    if (use_graph) ghip::rec_enable(g_dev[g_main_device].stream, false);
    const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    g_host_ns.fetch_add(ns, std::memory_order_relaxed);
    g_op_ns[t->op].fetch_add(ns, std::memory_order_relaxed);
    if (trace)
        fprintf(stderr, "node_ns %lld %lld\n", (long long)ns,
                (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count());
    return true;
}

int ggml_cpu_has_hipblas(void) {
    ensure_init();
    return g_device_count > 0 ? 1 : 0;
}

// ------------------------------------------------------------------------------------------
// tensor-free entry points

int ggml_hip_quantize_q8_0(const float *dev_x, int64_t K, int64_t N, void *dev_xq, void *stream) {
    if (!dev_x || !dev_xq || K <= 0 || K % QK || N < 0) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (!aligned(dev_x, 16) || !aligned(dev_xq, 2)) return fail(GGML_HIP_ERR_INVALID, "x must be 16-byte aligned");
    HIP_RET(ghip::quantize_q8_0_aos(dev_x, K, N, dev_xq, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_quantize_q4_0(const float *dev_w, int64_t K, int64_t M, void *dev_wq, void *stream) {
    if (!dev_w || !dev_wq || K <= 0 || K % QK || M < 0) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (!aligned(dev_w, 16) || !aligned(dev_wq, 2)) return fail(GGML_HIP_ERR_INVALID, "w must be 16-byte aligned");
    HIP_RET(ghip::quantize_q4_0(dev_w, K, M, dev_wq, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_dequantize_q4_0(const void *dev_wq, int64_t K, int64_t M, float *dev_w, void *stream) {
    if (!dev_w || !dev_wq || K <= 0 || K % QK || M < 0) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    HIP_RET(ghip::dequantize_q4_0(dev_wq, K, M, dev_w, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_mul_mat_q4_0(const void *dev_w, int64_t K, int64_t M, const float *dev_x, int64_t N, float *dev_y,
                          void *stream) {
    ensure_init();
    return mul_mat_dev(dev_w, K, M, dev_x, N, dev_y, M, 0, resolve_stream(stream));
}

int ggml_hip_mul_mat_q4_0_ex(const void *dev_w, int64_t K, int64_t M, const float *dev_x, int64_t N, float *dev_y,
                             int64_t ldy, int algo, void *stream) {
    ensure_init();
    return mul_mat_dev(dev_w, K, M, dev_x, N, dev_y, ldy, algo, resolve_stream(stream));
}

int ggml_hip_mul_mat_q4_0_multi(int n, const void *const *dev_w, const int64_t *M, int64_t K, const float *dev_x,
                                int64_t N, float *const *dev_y, void *stream) {
    ensure_init();
    if (n < 1 || n > ghip::GEMV_MULTI_MAX || !dev_w || !M || !dev_y)
        return fail(GGML_HIP_ERR_INVALID, "n must be 1..4 with non-null arrays");
    hipStream_t s = resolve_stream(stream);
    int64_t total = 0;
    for (int i = 0; i < n; i++) {
        if (!dev_w[i] || !dev_y[i] || M[i] <= 0) return fail(GGML_HIP_ERR_INVALID, "null matrix or M <= 0");
        if (!aligned(dev_w[i], 16) || !aligned(dev_y[i], 4)) return fail(GGML_HIP_ERR_INVALID, "misaligned W or y");
        total += M[i];
    }
    if (N == 0) return GGML_HIP_OK;
    if (exact_mode() && n > 1 && N >= 1 && dev_x && K > 0 && K % 64 == 0 && aligned(dev_x, 16) && total < (1 << 30)) {
        // exact mode: x quantized once, every sibling in ONE exact launch (bitwise the same as one
        // launch per matrix: each output row's chain does not depend on the grid)
        for (int i = 0; i < n; i++)
            if (M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31)) return fail(GGML_HIP_ERR_UNSUPPORTED, "matrix too large");
        const int id = current_device();
        void *ws = nullptr;
        const int wrc = stream_workspace(id, s, workspace_bytes(K, N), &ws);
        if (wrc != GGML_HIP_OK) return wrc;
        int8_t *qs = (int8_t *)ws;
        float *xd = (float *)((char *)ws + ((size_t)(N * K + 255) & ~(size_t)255));
        HIP_RET(ghip::quantize_q8_0_soa(dev_x, K, N, qs, xd, s));
        int64_t ldy[ghip::GEMV_MULTI_MAX];
        for (int i = 0; i < n; i++) ldy[i] = M[i];
        HIP_RET(ghip::mm_exact_q4_0_multi(n, dev_w, M, K, qs, xd, N, dev_y, ldy, s));
        return GGML_HIP_OK;
    }
    if (N > ghip::gemv_max_tokens(K) || total >= (1 << 30) || exact_mode()) {
        if (!exact_mode() && dev_x && K > 0 && K % 64 == 0) {
            // the image GEMMs' per-call weight image grows with M: size the workspace for the largest
            // sibling first, so that a later sibling cannot reallocate it under the shared q8_0 / x image
            // an earlier sibling left there.  At every N of the GEMM path: a tall sibling with an image
            // takes the image GEMM at any N above the GEMV's (IMG_MIN_M), next to split-K siblings
            int64_t mmax = 0;
            for (int i = 0; i < n; i++) mmax = std::max(mmax, M[i]);
            void *ws = nullptr;
            const int wrc = stream_workspace(current_device(), s, workspace_bytes_mm(K, N, mmax), &ws);
            if (wrc != GGML_HIP_OK) return wrc;
        }
        if (n > 1 && !exact_mode()) {
            const int rc = mul_mat_group_g9(n, dev_w, M, K, dev_x, N, dev_y, s);
            if (rc != 1) return rc;           // 1: not every sibling takes k_gemm9 on an fp6 image
        }
        unsigned xq = 0;
        for (int i = 0; i < n; i++) {       // GEMM / exact path: x quantized once, one launch per matrix
            int rc = mul_mat_dev(dev_w[i], K, M[i], dev_x, N, dev_y[i], M[i], 0, s, &xq);
            if (rc != GGML_HIP_OK) return rc;
        }
        return GGML_HIP_OK;
    }
    // validate the shared shape once through the single-matrix checks
    if (!dev_x || K <= 0 || K % 64 != 0 || !aligned(dev_x, 16)) return fail(GGML_HIP_ERR_INVALID, "bad x or K");
    for (int i = 0; i < n; i++)
        if (M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31)) return fail(GGML_HIP_ERR_UNSUPPORTED, "matrix too large");
    int64_t ldy[ghip::GEMV_MULTI_MAX];
    for (int i = 0; i < n; i++) ldy[i] = M[i];
    HIP_RET(ghip::gemv_q4_0_multi(n, dev_w, M, K, dev_x, N, dev_y, ldy, g_dev[current_device()].info, s));
    return GGML_HIP_OK;
}

int ggml_hip_set_exact(int on) {
    g_exact.store(on ? 1 : 0, std::memory_order_relaxed);
    return GGML_HIP_OK;
}

int ggml_hip_get_exact(void) { return exact_mode() ? 1 : 0; }

int ggml_hip_reserve_workspace(int64_t K, int64_t N) {
    ensure_init();
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    return reserve_workspace(current_device(), workspace_bytes(K, N));
}

int ggml_hip_weight_image_create(const void *dev_w, int64_t K, int64_t M, void *stream) {
    ensure_init();
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    if (!dev_w || K <= 0 || K % 64 != 0 || M <= 0 || !aligned(dev_w, 16))
        return fail(GGML_HIP_ERR_INVALID, "bad weight pointer or shape (K % 64 == 0, 16-byte aligned)");
    if (M * (K / QK) * Q4B >= ((int64_t)1 << 31) || (K / QK) * 2048 >= ((int64_t)1 << 31))
        return fail(GGML_HIP_ERR_UNSUPPORTED, "matrix too large");
    hipStream_t s = resolve_stream(stream);
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone)
        return fail(GGML_HIP_ERR_INVALID, "weight images are built outside stream capture");
    ghip::rec_flush_at("weight image");
    if (!wimage_ensure(current_device(), dev_w, K, M, s)) return fail(GGML_HIP_ERR_NOMEM, "weight image allocation failed");
    return GGML_HIP_OK;
}

int ggml_hip_weight_image_free(const void *dev_w) {
    ensure_init();
    ghip::rec_flush_at("weight image");
    return (int)wimage_drop(dev_w, 0);
}

int64_t ggml_hip_weight_image_bytes(void) {
    std::lock_guard<std::mutex> lk(g_wi_mu);
    return g_wi_resident;
}

int ggml_hip_debug_set_gemm_version(int v) {
    if (v != -1 && (v < 7 || v > 11)) return fail(GGML_HIP_ERR_INVALID, "version must be 7 ... 11 or -1");
    g_gemm_v.store(v, std::memory_order_relaxed);
    if (v == -1) (void)gemm_version();            // re-read GGML_HIP_GEMM_V
    return GGML_HIP_OK;
}

int ggml_hip_reserve_workspace_mm(int64_t K, int64_t N, int64_t M) {
    ensure_init();
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    if (K <= 0 || N < 0 || M < 0) return fail(GGML_HIP_ERR_INVALID, "bad shape");
    return reserve_workspace(current_device(), workspace_bytes_mm(K, N, M));
}

// ------------------------------------------------------------------------------------------
// decode chains: tasks validated once, launched as stream-ordered sibling GEMVs (one launch per task).
// Round 2 ran a chain as one persistent launch and round 4 as overlapped launches on two streams with
// per-workgroup flag hand-offs; both were bitwise equal and measured slower than one
// kernel per task (the in-launch hand-off costs more than a kernel boundary plus the GEMV's prologue),
// so a chain is the per-launch path.

}  // extern "C"

struct ggml_hip_chain {
    int device = 0;
    std::vector<ggml_hip_chain_task> tasks;
};

extern "C" {

int ggml_hip_chain_create(int ntasks, const ggml_hip_chain_task *tasks, ggml_hip_chain **out) {
    ensure_init();
    if (!out) return fail(GGML_HIP_ERR_INVALID, "null out");
    *out = nullptr;
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    if (ntasks < 1 || !tasks) return fail(GGML_HIP_ERR_INVALID, "ntasks must be >= 1");
    for (int t = 0; t < ntasks; t++) {
        const ggml_hip_chain_task &k = tasks[t];
        if (k.nmat < 1 || k.nmat > ghip::GEMV_MULTI_MAX) return fail(GGML_HIP_ERR_INVALID, "nmat must be 1..4");
        if (k.K <= 0 || k.K % 64 != 0 || !k.x || !aligned(k.x, 16))
            return fail(GGML_HIP_ERR_INVALID, "bad x or K (K % 64 == 0, 16-byte aligned x)");
        for (int i = 0; i < k.nmat; i++) {
            if (!k.W[i] || !k.y[i] || k.M[i] <= 0 || !aligned(k.W[i], 16) || !aligned(k.y[i], 4))
                return fail(GGML_HIP_ERR_INVALID, "null / misaligned W or y, or M <= 0");
            // a task's y may not overlap its own x (its rows read x while others write y)
            const uint64_t xlo = (uint64_t)(uintptr_t)k.x, xhi = xlo + 4 * (uint64_t)k.K;
            const uint64_t yp = (uint64_t)(uintptr_t)k.y[i];
            if (yp < xhi && xlo < yp + 4 * (uint64_t)k.M[i]) return fail(GGML_HIP_ERR_INVALID, "a task's y overlaps its own x");
        }
    }
    auto *c = new ggml_hip_chain();
    c->device = current_device();
    c->tasks.assign(tasks, tasks + ntasks);
    *out = c;
    return GGML_HIP_OK;
}

int ggml_hip_chain_launch(ggml_hip_chain *c, void *stream) {
    ensure_init();
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null chain");
    if (current_device() != c->device) return fail(GGML_HIP_ERR_INVALID, "chain belongs to another device");
    hipStream_t s = resolve_stream(stream);
    for (const auto &k : c->tasks) {
        const int rc = ggml_hip_mul_mat_q4_0_multi(k.nmat, k.W, k.M, k.K, k.x, 1, (float *const *)k.y, s);
        if (rc != GGML_HIP_OK) return rc;
    }
    return GGML_HIP_OK;
}

int ggml_hip_chain_status(ggml_hip_chain *c) {
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null chain");
    HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());
    return 0;
}

int ggml_hip_chain_destroy(ggml_hip_chain *c) {
    delete c;
    return GGML_HIP_OK;
}

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

}  // extern "C"

namespace {

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

}  // namespace

struct ggml_hip_comm {
    ncclComm_t comm = nullptr;
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
    uint32_t *p2p_herr = nullptr;     // host-mapped error word the gather kernel sets on a timeout
    double p2p_timeout_ms = -1.0;     // < 0: GGML_HIP_P2P_TIMEOUT_MS (default 10000)
    // file rendezvous transport (ggml_hip_comm_init_file): host collectives through files in fdir
    std::string fdir;
    uint64_t fseq = 0;
};

namespace {

#define NCCL_RET(expr)                                                                               \
    do {                                                                                             \
        ncclResult_t r_ = (expr);                                                                    \
        if (r_ != ncclSuccess) {                                                                     \
            g_last_error = std::string(#expr) + ": " + ncclGetErrorString(r_);                       \
            return GGML_HIP_ERR_COMM;                                                                \
        }                                                                                            \
    } while (0)

// file rendezvous: rank r writes <dir>/c<seq>_r<r> (tmp + rename), then reads every rank's file of the
// same sequence number; a rank that sees all R files of seq knows every rank finished reading seq - 1,
// so it removes its own file of seq - 1.  Bounded wait (GGML_HIP_COMM_FILE_TIMEOUT_S, default 120 s).
int file_allgather(ggml_hip_comm *c, const void *mine, size_t n, std::vector<char> &all) {
    const uint64_t seq = c->fseq++;
    auto name = [&](uint64_t s, int r) { return c->fdir + "/c" + std::to_string(s) + "_r" + std::to_string(r); };
    const std::string me = name(seq, c->rank);
    {
        FILE *f = fopen((me + ".tmp").c_str(), "wb");
        if (!f) return fail(GGML_HIP_ERR_COMM, "file comm: cannot write " + me);
        const bool ok = fwrite(mine, 1, n, f) == n;
        if (fclose(f) != 0 || !ok) return fail(GGML_HIP_ERR_COMM, "file comm: short write " + me);
        if (rename((me + ".tmp").c_str(), me.c_str()) != 0) return fail(GGML_HIP_ERR_COMM, "file comm: rename " + me);
    }
    static const double limit_s = getenv("GGML_HIP_COMM_FILE_TIMEOUT_S") ? atof(getenv("GGML_HIP_COMM_FILE_TIMEOUT_S")) : 120.0;
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
    else if (GHIP_SYNC(ncclAllGather)(dev + n * c->rank, dev, n, ncclChar, c->comm, s) != ncclSuccess)
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
    if (p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: a peer wait timed out earlier; the comm is failed");
    if (c->transport == 1 && c->p2p_on && (int64_t)count <= c->p2p.cap) {
        HIP_RET(ghip::p2p_allgather(c->p2p, send, (int64_t)count, recv, s));
        return GGML_HIP_OK;
    }
    if (!c->fdir.empty()) return fail(GGML_HIP_ERR_UNSUPPORTED, "file comm: device all-gathers need the P2P transport");
    if (!c->local) {
        NCCL_RET(GHIP_SYNC(ncclAllGather)(send, recv, count, ncclFloat32, c->comm, s));
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
    if (c->comm && c->transport == 0) NCCL_RET(GHIP_SYNC(ncclGroupEnd)());
    return GGML_HIP_OK;
}

}  // namespace

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
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(GGML_HIP_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
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
    *comm = c;
    return GGML_HIP_OK;
}

int ggml_hip_comm_destroy(ggml_hip_comm *c) {
    if (!c) return GGML_HIP_OK;
    if (c->p2p_on) (void)GHIP_SYNC(hipDeviceSynchronize)();
    for (void *p : c->p2p_opened) (void)hipIpcCloseMemHandle(p);
    if (c->p2p_mine) (void)GHIP_SYNC(hipFree)(c->p2p_mine);
    if (c->p2p_herr) (void)hipHostFree(c->p2p_herr);
    if (c->comm) ncclCommDestroy(c->comm);
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
    NCCL_RET(GHIP_SYNC(ncclAllReduce)(c->red_dev, c->red_dev, (size_t)n, ncclFloat64, ops[op], c->comm, s));
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
    if (hipHostMalloc((void **)&c->p2p_herr, 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        c->p2p_herr = nullptr;
        local_fail(GGML_HIP_ERR_NOMEM, "P2P host error word");
    } else {
        *c->p2p_herr = 0;
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
        if (grc != GGML_HIP_OK) return grc;   // the transport itself failed: no further collective can run
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
    c->p2p_timeout_ms = ms;
    c->p2p.timeout = (uint64_t)(ms * 1e5);     // s_memrealtime: 100 MHz
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
    uint64_t err = 0;
    HIP_RET(GHIP_SYNC(hipMemcpy)(&err, c->p2p.ctl + 2, 8, hipMemcpyDeviceToHost));
    return (int)err;                           // sticky: a failed comm stays failed
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
    if (p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: a peer wait timed out earlier; the comm is failed");
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
    if (c && p2p_failed(c)) return fail(GGML_HIP_ERR_COMM, "P2P all-gather: a peer wait timed out earlier; the comm is failed");
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

int ggml_hip_weight_cache_stats(int64_t *hits, int64_t *misses, int64_t *resident_bytes) {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    if (hits) *hits = (int64_t)g_wc_hits;
    if (misses) *misses = (int64_t)g_wc_misses;
    if (resident_bytes) *resident_bytes = (int64_t)g_wc_resident;
    return GGML_HIP_OK;
}

int ggml_hip_weight_cache_clear(void) {
    ensure_init();
    std::lock_guard<std::mutex> lk(g_wc_mu);
    for (int id = 0; id < g_device_count; id++) {
        HIP_RET(hipSetDevice(id));
        HIP_RET(GHIP_SYNC(hipStreamSynchronize)(g_dev[id].stream));
    }
    for (auto &e : g_wc) {
        wimage_drop(e.second.dev, e.second.bytes);
        HIP_RET(GHIP_SYNC(hipFree)(e.second.dev));
    }
    g_wc.clear();
    g_wc_resident = 0;
    g_wc_hits = g_wc_misses = g_wc_invalidations = 0;
    g_wc_lo.store(UINTPTR_MAX);
    g_wc_hi.store(0);
    return GGML_HIP_OK;
}

int64_t ggml_hip_weight_cache_invalidate(const void *host, size_t bytes) {
    if (!host) return GGML_HIP_ERR_INVALID;
    flush_deferred();
    return wcache_invalidate(host, bytes);
}

int ggml_hip_weight_cache_set_verify(int mode) {
    if (mode < -1 || mode > 1) return fail(GGML_HIP_ERR_INVALID, "verify mode must be -1, 0 or 1");
    g_wc_verify_override.store(mode);
    return GGML_HIP_OK;
}

int64_t ggml_hip_weight_cache_invalidations(void) {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    return (int64_t)g_wc_invalidations;
}

// ------------------------------------------------------------------------------------------
// device plumbing

int ggml_hip_device_count(void) {
    ensure_init();
    return g_device_count;
}

int ggml_hip_set_device(int device) {
    ensure_init();
    HIP_RET(hipSetDevice(device));
    return GGML_HIP_OK;
}

int ggml_hip_get_device(void) { return current_device(); }

void *ggml_hip_dev_malloc(size_t size) {
    ensure_init();
    void *p = nullptr;
    if (hipMalloc(&p, size ? size : 1) != hipSuccess) {
        (void)hipGetLastError();
        g_last_error = "hipMalloc failed";
        return nullptr;
    }
    return p;
}

void ggml_hip_dev_free(void *ptr) {
    if (ptr) (void)GHIP_SYNC(hipFree)(ptr);
}

int ggml_hip_memcpy_h2d(void *dst, const void *src, size_t size, void *stream) {
    flush_deferred();
    hipStream_t s = resolve_stream(stream);
    HIP_RET(GHIP_SYNC(hipMemcpyAsync)(dst, src, size, hipMemcpyHostToDevice, s));
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_memcpy_d2h(void *dst, const void *src, size_t size, void *stream) {
    flush_deferred();
    hipStream_t s = resolve_stream(stream);
    HIP_RET(GHIP_SYNC(hipMemcpyAsync)(dst, src, size, hipMemcpyDeviceToHost, s));
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_memcpy_d2d(void *dst, const void *src, size_t size, void *stream) {
    flush_deferred();
    HIP_RET(GHIP_SYNC(hipMemcpyAsync)(dst, src, size, hipMemcpyDeviceToDevice, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_memset(void *dst, int value, size_t size, void *stream) {
    HIP_RET(GHIP_SYNC(hipMemsetAsync)(dst, value, size, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_stream_synchronize(void *stream) {
    flush_deferred();
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_device_synchronize(void) {
    flush_deferred();
    HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());
    return GGML_HIP_OK;
}

void *ggml_hip_default_stream(void) { return (void *)resolve_stream(nullptr); }

void *ggml_hip_stream_create(void) {
    ensure_init();
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        g_last_error = "hipStreamCreateWithFlags failed";
        return nullptr;
    }
    return (void *)s;
}

int ggml_hip_stream_destroy(void *stream) {
    if (!stream) return GGML_HIP_OK;
    hipStream_t s = (hipStream_t)stream;
    HIP_RET(GHIP_SYNC(hipStreamSynchronize)(s));
    for (int id = 0; id < g_device_count; id++) {
        Device &d = g_dev[id];
        std::lock_guard<std::mutex> lk(d.mu);
        auto it = d.stream_ws.find(s);
        if (it != d.stream_ws.end()) {
            if (it->second.ptr) HIP_RET(GHIP_SYNC(hipFree)(it->second.ptr));
            d.stream_ws.erase(it);
        }
    }
    HIP_RET(GHIP_SYNC(hipStreamDestroy)(s));
    return GGML_HIP_OK;
}

int ggml_hip_fill_gaussian(float *dev_dst, int64_t n, uint64_t seed, float mean, float stdv, void *stream) {
    HIP_RET(ghip::fill_gaussian(dev_dst, n, seed, mean, stdv, resolve_stream(stream)));
    return GGML_HIP_OK;
}

void *ggml_hip_event_create(void) {
    ensure_init();
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return (void *)e;
}

int ggml_hip_event_record(void *event, void *stream) {
    HIP_RET(GHIP_SYNC(hipEventRecord)((hipEvent_t)event, resolve_stream(stream)));
    return GGML_HIP_OK;
}

float ggml_hip_event_elapsed_ms(void *start, void *stop) {
    float ms = -1.0f;
    hipError_t e = GHIP_SYNC(hipEventSynchronize)((hipEvent_t)stop);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, (hipEvent_t)start, (hipEvent_t)stop);
    if (e != hipSuccess) {
        (void)hipGetLastError();      // do not leave a sticky error for the next launch check
        g_last_error = std::string("hipEventElapsedTime: ") + hipGetErrorString(e);
        return -1.0f;
    }
    return ms;
}

void ggml_hip_event_destroy(void *event) {
    if (event) (void)hipEventDestroy((hipEvent_t)event);
}

struct ggml_hip_graph {
    hipGraph_t graph;
    hipGraphExec_t exec;
};

int ggml_hip_graph_begin(void *stream) {
    HIP_RET(GHIP_SYNC(hipStreamBeginCapture)(resolve_stream(stream), hipStreamCaptureModeThreadLocal));
    return GGML_HIP_OK;
}

int ggml_hip_graph_end(void *stream, ggml_hip_graph **out) {
    if (!out) return fail(GGML_HIP_ERR_INVALID, "null graph out");
    auto *g = new ggml_hip_graph;
    HIP_RET(GHIP_SYNC(hipStreamEndCapture)(resolve_stream(stream), &g->graph));
    HIP_RET(hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0));
    *out = g;
    return GGML_HIP_OK;
}

int ggml_hip_graph_launch(ggml_hip_graph *g, void *stream) {
    if (!g) return fail(GGML_HIP_ERR_INVALID, "null graph");
    HIP_RET(GHIP_SYNC(hipGraphLaunch)(g->exec, resolve_stream(stream)));
    return GGML_HIP_OK;
}

int ggml_hip_graph_destroy(ggml_hip_graph *g) {
    if (!g) return GGML_HIP_OK;
    (void)hipGraphExecDestroy(g->exec);
    (void)hipGraphDestroy(g->graph);
    delete g;
    return GGML_HIP_OK;
}

const char *ggml_hip_last_error(void) { return g_last_error.c_str(); }

// not in the public header: tests force each GEMV launch policy (all must give the same y)
int ggml_hip_debug_set_gemv_policy(int map, int depth, int rowitems, int wg_per_cu) {
    if (map < -1 || map > 2 || depth < 0 || depth > 2 || rowitems < 0 || rowitems > 1 || wg_per_cu < 0)
        return fail(GGML_HIP_ERR_INVALID, "bad GEMV policy");
    ghip::gemv_set_policy(map, depth, rowitems, wg_per_cu);
    return GGML_HIP_OK;
}

// not in the public header: the chunk-balanced decode GEMV (BAL) for K > 12288: -1 auto, 0 off, 1 on
int ggml_hip_debug_set_gemv_bal(int bal) {
    if (bal < -1 || bal > 1) return fail(GGML_HIP_ERR_INVALID, "bad GEMV balance mode");
    ghip::gemv_set_bal(bal);
    return GGML_HIP_OK;
}

// not in the public header: the smallest host Q4_0 weight (elements) taken at N < 32 through the
// residency cache (-1 = GGML_HIP_DECODE_MIN_WEIGHTS or 2^19); returns the previous value
int64_t ggml_hip_debug_set_decode_min_weights(int64_t n) {
    const int64_t prev = decode_min_weights();
    g_decode_min_weights.store(n < 0 ? -1 : n);
    return prev;
}

// not in the public header: nodes taken by ggml_hip_compute_forward per ggml op (counts[op], op < n);
// reset when reset != 0 (tests check which ops of a full-offload graph ran on the device)
int ggml_hip_debug_op_stats(int64_t *counts, int n, int reset) {
    for (int i = 0; i < n && i < gabi::OP_COUNT; i++) counts[i] = g_op_count[i].load();
    if (n > gabi::OP_COUNT) counts[gabi::OP_COUNT] = g_host_ns.load();   // one slot past the ops: host ns
    for (int i = 0; i < gabi::OP_COUNT && gabi::OP_COUNT + 1 + i < n; i++) counts[gabi::OP_COUNT + 1 + i] = g_op_ns[i].load();
    for (int i = 0; i < N_FUSED && 2 * gabi::OP_COUNT + 1 + i < n; i++) counts[2 * gabi::OP_COUNT + 1 + i] = g_fused[i].load();
    if (reset) {
        for (auto &c : g_op_count) c.store(0);
        for (auto &c : g_fused) c.store(0);
        for (auto &c : g_op_ns) c.store(0);
        g_host_ns.store(0);
    }
    return GGML_HIP_OK;
}

// not in the public header: launch-recorder counters (launch.h) — out[0] submitted runs, [1] kernels in
// them, [2] graph nodes updated in place, [3] graphs instantiated, [4] host ns spent submitting;
// clear != 0 also destroys the cache
int ggml_hip_debug_graph_stats(long long *out, int clear) {
    flush_deferred();
    ghip::rec_stats(&out[0], &out[1], &out[2], &out[3], &out[4]);
    if (clear) ghip::rec_clear_cache();
    return GGML_HIP_OK;
}

// not in the public header: the decode norm chain folded into the GEMV prologue on (1) / off (0)
int ggml_hip_debug_set_norm_fold(int on) {
    flush_deferred();
    g_norm_fold.store(on < 0 || on > 2 ? 1 : on);
    return GGML_HIP_OK;
}

// not in the public header: the prefill x image fold (a held norm / silu chain writes the k_gemm9 x image
// of its output for the q4_0 mul_mats that consume it) on (1) / off (0)
int ggml_hip_debug_set_x9_fold(int on) {
    flush_deferred();
    g_x9_fold.store(on ? 1 : 0);
    return GGML_HIP_OK;
}

// not in the public header: launch recording for the hook path: 0 off, 1 HIP graphs, 2 launcher thread
int ggml_hip_debug_set_graph(int on) {
    flush_deferred();
    graph_flag().store(on);
    return GGML_HIP_OK;
}

// debug (tests/test_gpu_parity.py::test_x9_producers_bitwise): the prefill chains that write the k_gemm9 x
// image of their output (kind 1: [a + b ->] rms_norm -> * w, a may be null; kind 2: u = silu(a) -> u * b)
// into img, the same chain without the image into out_ref, and gemm9_prep_x of out into img_ref
// (synchronous; images of gemm9 x-image size for ncols x nrows, zeroed by the caller)
int ggml_hip_debug_x9_producer(int kind, const float *a, const float *b, const float *w, float *sum, float *norm,
                               float *out, float *out_ref, int64_t ncols, int64_t nrows, void *img, void *img_ref) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    if ((kind != 1 && kind != 2) || !ghip::op_x9_ok(ncols, nrows)) return fail(GGML_HIP_ERR_INVALID, "bad x9 producer");
    flush_deferred();
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    hipStream_t s = g_dev[id].stream;
    const int64_t Np = ghip::gemm9_np(nrows);
    if (kind == 1) {
        HIP_RET(ghip::op_add_rms_norm_mul_f32_x9(a, b, sum, norm, w, out, ncols, nrows, img, Np, s));
        HIP_RET(ghip::op_add_rms_norm_mul_f32(a, b, nullptr, nullptr, w, out_ref, ncols, nrows, s));
    } else {
        const OpTables &tb = op_tables(id, s);
        HIP_RET(ghip::op_silu_mul_f32_x9(a, b, norm, out, ncols, nrows, tb.silu, img, Np, s));
        HIP_RET(ghip::op_silu_mul_f32(a, b, nullptr, out_ref, ncols * nrows, tb.silu, s));
    }
    HIP_RET(ghip::gemm9_prep_x(out, ncols, nrows, img_ref, s));
    HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

// debug: the f16 x f32 mul_mat of the attention on device pointers (tests/test_gpu_f16_mul_mat.py):
// tiled 0 = one 32-lane group per output, 1 = the LDS-tiled kernel, -1 = the backend's choice (bitwise
// kernels), 2 = the fast-mode MFMA kernel, -2 = the backend's fast-mode choice
int ggml_hip_debug_f16_mul_mat(const void *s0, const void *s1, float *d, int K, int64_t ne01, int64_t ne11,
                               int64_t ne02, int64_t nb01, int64_t nb02, int64_t nb11, int64_t nb12, float *merged,
                               int tiled) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    flush_deferred();
    HIP_FATAL(hipSetDevice(g_main_device));
    hipStream_t s = g_dev[g_main_device].stream;
    HIP_FATAL(ghip::op_mul_mat_f16_f32(s0, s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12, s, merged, tiled));
    HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_debug_rope(const void *x, void *d, void *c, int to_f16, int64_t ne0, int64_t ne1, int64_t ne2, int n_past,
                        int n_dims, const int64_t *nbx, const int64_t *nbd, int64_t ne10, int64_t ne11, int64_t nb10,
                        int64_t nb11, int64_t nb12, int batched) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    if (ne0 < 2 || ne0 % 2 || ne1 < 1 || ne2 < 1 || n_past < 0 || n_dims < 2 || n_dims % 2 || n_dims > ne0 || !nbx || !nbd)
        return GGML_HIP_ERR_INVALID;
    flush_deferred();
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    hipStream_t s = g_dev[id].stream;
    const int64_t np = ne0 / 2;
    const float *cs = rope_table(id, ne0, n_dims, (int64_t)n_past + ne2, s) + (size_t)n_past * np * 2;
    const int64_t ne[4] = {ne0, ne1, ne2, 1};
    if (batched) {
        ghip::ElemBatch b{};
        ghip::ElemOp &op = b.op[0];
        op.kind = 0;
        op.x = (const char *)x;
        op.d = (char *)d;
        op.cs = (const float2 *)cs;
        op.npairs = (int)np;
        op.n = np * ne1 * ne2;
        op.ne0 = ne0, op.ne1 = ne1, op.ne2 = ne2;
        op.nbx1 = nbx[1], op.nbx2 = nbx[2], op.nbx3 = nbx[3];
        op.nbd1 = nbd[1], op.nbd2 = nbd[2], op.nbd3 = nbd[3];
        if (c) {
            op.c = (char *)c;
            op.f16 = to_f16 != 0;
            op.ne10 = ne10, op.ne11 = ne11, op.nb10 = nb10, op.nb11 = nb11, op.nb12 = nb12;
        }
        b.nops = 1;
        HIP_FATAL(ghip::op_elem_batch(b, s));
    } else if (c) {
        HIP_FATAL(ghip::op_rope_cpy_f32(x, d, ne, nbx, nbd, cs, (int)np, c, to_f16 != 0, ne10, ne11, nb10, nb11, nb12, s));
    } else {
        HIP_FATAL(ghip::op_rope_f32(x, d, ne, nbx, nbd, cs, (int)np, s));
    }
    HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

int ggml_hip_debug_cpy_f32(const void *x, void *d, int to_f16, int64_t n, int64_t ne00, int64_t ne01, int64_t nb00,
                           int64_t nb01, int64_t nb02, int64_t ne10, int64_t ne11, int64_t nb10, int64_t nb11,
                           int64_t nb12, int batched) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    if (n < 0 || ne00 < 1 || ne01 < 1 || ne10 < 1 || ne11 < 1) return GGML_HIP_ERR_INVALID;
    flush_deferred();
    HIP_FATAL(hipSetDevice(g_main_device));
    hipStream_t s = g_dev[g_main_device].stream;
    if (batched) {
        ghip::ElemBatch b{};
        ghip::ElemOp &op = b.op[0];
        op.kind = 1, op.f16 = to_f16 != 0, op.x = (const char *)x, op.c = (char *)d, op.n = n;
        op.ne0 = ne00, op.ne1 = ne01, op.nbx1 = nb00, op.nbx2 = nb01, op.nbx3 = nb02;
        op.ne10 = ne10, op.ne11 = ne11, op.nb10 = nb10, op.nb11 = nb11, op.nb12 = nb12;
        b.nops = 1;
        HIP_FATAL(ghip::op_elem_batch(b, s));
    } else {
        HIP_FATAL(ghip::op_cpy_f32(x, d, to_f16 != 0, n, ne00, ne01, nb00, nb01, nb02, ne10, ne11, nb10, nb11, nb12, s));
    }
    HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

// not in the public header: launch fusion of full-offload chains on (1) / off (0) (tests run both)
int ggml_hip_debug_set_fuse(int on) {
    flush_deferred();
    g_fuse.store(on ? 1 : 0, std::memory_order_relaxed);
    return GGML_HIP_OK;
}

const char *ggml_hip_version(void) { return "ggml-hip q4_0 gfx950 r1"; }

}  // extern "C"
