// ggml-hip-wcache.cpp — the device copies of weights: prefill weight images (int8 / fp6, built once per
// weight) and the residency cache for CPU-backend Q4_0 weights.
#include "ggml-hip-internal.h"

using namespace ghh;

namespace ghh {

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
std::mutex g_wi_mu;
std::map<std::pair<int, uintptr_t>, WImage> g_wi;          // (device, weight address)
int64_t g_wi_resident = 0;

const void *wimage_find(int id, const void *w, int64_t K, int64_t M, int *fmt) {
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

}  // namespace ghh

namespace ghh {

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

}  // namespace ghh

namespace ghh {

std::unordered_map<WCacheKey, WCacheEntry, WCacheHash> g_wc;
size_t g_wc_resident = 0;
uint64_t g_wc_clock = 0, g_wc_hits = 0, g_wc_misses = 0, g_wc_invalidations = 0;
std::atomic<uintptr_t> g_wc_lo{UINTPTR_MAX}, g_wc_hi{0};   // hull of the cached host ranges (monotone)

uint64_t wcache_next_call_id() {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    return ++g_wc_clock;
}

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

// LRU eviction (g_wc_mu held) until `incoming` more bytes fit the budget; entries used by the current
// call (last_use == call_id) are never evicted (a kernel of this call may read them)
void wcache_evict_locked(size_t incoming, uint64_t call_id) {
    while (g_wc_resident + incoming > wcache_budget()) {
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
    wcache_evict_locked(bytes, call_id);
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
void wcache_note_image(int id, const void *dev, size_t img_bytes, uint64_t call_id) {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    for (auto &e : g_wc)
        if (e.first.device == id && e.second.dev == dev && e.second.img_bytes == 0) {
            e.second.img_bytes = img_bytes;
            g_wc_resident += img_bytes;
            wcache_evict_locked(0, call_id);           // back under the budget now, not at the next miss
            return;
        }
}

// ggml_hip_weight_image_free dropped the image at dev: a cached copy there no longer carries its bytes
void wcache_image_dropped(const void *dev) {
    std::lock_guard<std::mutex> lk(g_wc_mu);
    for (auto &e : g_wc)
        if (e.second.dev == dev && e.second.img_bytes) {
            g_wc_resident -= e.second.img_bytes;
            e.second.img_bytes = 0;
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

}  // namespace ghh

extern "C" {

int64_t ggml_hip_weight_image_bytes(void) {
    std::lock_guard<std::mutex> lk(g_wi_mu);
    return g_wi_resident;
}

}  // extern "C"

extern "C" {

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

}  // extern "C"

extern "C" {

// not in the public header: the smallest host Q4_0 weight (elements) taken at N < 32 through the
// residency cache (-1 = GGML_HIP_DECODE_MIN_WEIGHTS or 2^19); returns the previous value
int64_t ggml_hip_debug_set_decode_min_weights(int64_t n) {
    const int64_t prev = decode_min_weights();
    g_decode_min_weights.store(n < 0 ? -1 : n);
    return prev;
}

}  // extern "C"
