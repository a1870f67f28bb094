// ggml-hip-core.cpp — host side of the MI355X q4_0 mul_mat backend: per-device state, temporaries,
// workspaces and the device-pointer mul_mat core (ggml_compute_forward_mul_mat_q_f32 INIT + COMPUTE).
// The C ABI of include/ggml-hip.h is spread over ggml-hip-{api,tensor,fuse,ops,wcache,comm}.cpp, which
// share the declarations of ggml-hip-internal.h.  Mirrors the reference's ggml-cuda.cu host plumbing for
// this path (file:line in each function comment) with a native design:
//   * one non-blocking HIP stream per device, created once (ggml-cuda.cu:1849);
//   * a per-device caching pool for temporaries (ggml-cuda.cu:1751-1811);
//   * mul_mat = fused q8_0-quantize + GEMV for N <= 8 tokens, q8_0-quantize + MFMA GEMMs otherwise
//     (replacing dequantize_mul_mat_vec / dequantize_block + cublasSgemm, ggml-cuda.cu:1177-1244,
//     1156-1175, 2143-2182).
#include "ggml-hip-internal.h"

using namespace ghh;

namespace ghh {

// ------------------------------------------------------------------------------------------
// errors: the tensor ABI is fail-fast like CUDA_CHECK (ggml-cuda.cu:22-51); the tensor-free
// ABI returns a status and keeps the message for ggml_hip_last_error().

thread_local std::string g_last_error;

}  // namespace ghh

namespace ghh {

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

}  // namespace ghh

namespace ghh {

std::once_flag g_init_once;
int g_device_count = 0;
Device *g_dev = nullptr;
int g_main_device = 0;
float g_tensor_split[GGML_HIP_MAX_DEVICES] = {0};

}  // namespace ghh

namespace ghh {

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

void ensure_init() { std::call_once(g_init_once, init_impl); }

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

}  // namespace ghh

namespace ghh {

int reserve_workspace(int id, size_t bytes, hipStream_t s) {
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

}  // namespace ghh

namespace ghh {

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
int mul_mat_dev(const void *w, int64_t K, int64_t M, const float *x, int64_t N, float *y, int64_t ldy, int algo,
                hipStream_t s, unsigned *xq) {
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
// row tiles (the x image built once, as before).  The launch plans its tiles (128 x 128 / 128 x 64 /
// mixed, half tiles) from its own total tile count, which can differ from the per-matrix launches'
// plans: y is within the oracle bound of the separate calls, and bitwise equal to them only with the
// tile pinned (ggml_hip_debug_set_gemm9_wide 0 or 1; include/ggml-hip.h).
// Returns 1 when the group does not qualify (the caller runs one launch per matrix).
bool g9_images(int n, const void *const *w, const int64_t *M, int64_t K, int64_t N, const void **img) {
    static const bool grp = !getenv("GGML_HIP_GEMM9_GROUP") || atoi(getenv("GGML_HIP_GEMM9_GROUP")) != 0;
    if ((n > 1 && !grp) || n < 1 || n > 4 || exact_mode() || gemm_version() != 10 || K <= 0 || K % 64 != 0 ||
        N <= ghip::gemv_max_tokens(K) || N * K >= ((int64_t)1 << 31))
        return false;
    const int id = current_device();
    for (int i = 0; i < n; i++) {
        int fmt = 0;
        img[i] = wimage_find(id, w[i], K, M[i], &fmt);
        // mul_mat_dev's algo rule: the image GEMM above 128 tokens, or above IMG_MIN_N / for tall
        // matrices when an image exists
        if (!img[i] || fmt != 9 || !(N > 128 || N > IMG_MIN_N || M[i] >= IMG_MIN_M)) return false;
        if (M[i] * (K / QK) * Q4B >= ((int64_t)1 << 31) || M[i] >= (1 << 30)) return false;
    }
    return true;
}

int mul_mat_group_g9(int n, const void *const *w, const int64_t *M, int64_t K, const float *x, int64_t N,
                     float *const *y, hipStream_t s) {
    const void *img[4];
    if (n < 2 || !x || !aligned(x, 16) || !g9_images(n, w, M, K, N, img)) return 1;
    const int id = current_device();
    int64_t ldy[4];
    for (int i = 0; i < n; i++) ldy[i] = M[i];
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

}  // namespace ghh
