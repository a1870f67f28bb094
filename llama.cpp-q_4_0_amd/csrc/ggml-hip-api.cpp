// ggml-hip-api.cpp — the tensor-free C ABI on device pointers (quantizers, mul_mat, sibling batches, decode
// chains, weight images) and the device plumbing the bindings use (streams, events, graphs, copies).
#include "ggml-hip-internal.h"

using namespace ghh;

extern "C" {

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
    const int64_t n = wimage_drop(dev_w, 0);
    if (n) wcache_image_dropped(dev_w);
    return (int)n;
}

}  // extern "C"

extern "C" {

int ggml_hip_debug_set_gemm_version(int v) {
    if (v != -1 && (v < 7 || v > 11)) return fail(GGML_HIP_ERR_INVALID, "version must be 7 ... 11 or -1");
    g_gemm_v.store(v, std::memory_order_relaxed);
    if (v == -1) (void)gemm_version();            // re-read GGML_HIP_GEMM_V
    return GGML_HIP_OK;
}

int ggml_hip_debug_set_gemm9_wide(int mode) {
    if (mode < -1 || mode > 1) return fail(GGML_HIP_ERR_INVALID, "mode must be -1, 0 or 1");
    ghip::gemm9_set_wide(mode);
    return GGML_HIP_OK;
}

int ggml_hip_reserve_workspace_mm(int64_t K, int64_t N, int64_t M) {
    ensure_init();
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    if (K <= 0 || N < 0 || M < 0) return fail(GGML_HIP_ERR_INVALID, "bad shape");
    return reserve_workspace(current_device(), workspace_bytes_mm(K, N, M));
}

// ------------------------------------------------------------------------------------------
// decode chains: tasks validated once, launched as stream-ordered sibling GEMVs (one launch per task), or
// (ggml_hip_chain_set_engine / GGML_HIP_CHAIN_ENGINE) as ONE launch of the persistent LDS-DMA decode engine
// (q4_0_engine.hip), bitwise the same y.  Round 2 ran a chain as one persistent launch and round 4 as
// overlapped launches on two streams with per-workgroup flag hand-offs; both were bitwise
// equal and slower than one kernel per task.  The engine differs in what those lacked: one loader wave per
// CU streams the weights by LDS-DMA ahead across the edges, and an edge moves q8_0 granules quantized once.

}  // extern "C"

struct ggml_hip_chain {
    int device = 0;
    int64_t N = 1;                    // tokens per task (ggml_hip_chain_create_n)
    std::vector<ggml_hip_chain_task> tasks;
    ghip::EnginePlan *eng = nullptr;  // the engine's plan when the chain runs on it
    int eng_mode = 0;                 // 0 per-launch, 1 engine requested
    std::string eng_why;              // why the engine declined the chain (empty when it runs)
    // N > gemv tokens: per task, its k_gemm9 x image (gemm9_x_bytes(K, N)) and the task whose launch writes it
    // in its epilogue (-1: none, the task builds it with k_prep9_x); per task, the image its epilogue writes
    // (null: none) from the y of matrix out_mat.  Consumers of one producer's output share its image.
    std::vector<void *> ximg, out_img, owned;
    std::vector<int> prod_task, out_mat;
};

namespace {
int engine_env() {
    const char *e = getenv("GGML_HIP_CHAIN_ENGINE");
    return e ? atoi(e) : 0;
}
uint32_t engine_timeout_ticks() {       // s_memrealtime ticks (100 MHz); GGML_HIP_ENGINE_TIMEOUT_MS, default 2 s
    const char *e = getenv("GGML_HIP_ENGINE_TIMEOUT_MS");
    double ms = e ? atof(e) : 2000.0;
    if (!(ms > 0.0)) ms = 2000.0;
    if (ms > 40000.0) ms = 40000.0;     // fits 32 bits of ticks
    return (uint32_t)(ms * 1e5);
}
int chain_engine_on(ggml_hip_chain *c) {
    if (c->eng) return 1;
    c->eng_why.clear();
    if (c->N != 1) {
        c->eng_why = "the decode engine runs N = 1 chains";
        return 0;
    }
    const int ncu = g_dev[c->device].info.num_cus;
    c->eng = ghip::engine_plan_create((int)c->tasks.size(), c->tasks.data(), ncu, engine_timeout_ticks(), c->eng_why);
    return c->eng ? 1 : 0;
}
}  // namespace

extern "C" {

}  // extern "C"

namespace {
bool overlaps(const void *a, uint64_t abytes, const void *b, uint64_t bbytes) {
    const uint64_t p = (uint64_t)(uintptr_t)a, q = (uint64_t)(uintptr_t)b;
    return p < q + bbytes && q < p + abytes;
}

void chain_free_images(ggml_hip_chain *c) {
    for (void *p : c->owned) (void)hipFree(p);
    c->owned.clear();
    c->ximg.clear();
    c->out_img.clear();
}

// The image plan of an N-token chain.  Task t's producer is the latest earlier task u with a matrix i whose y
// is exactly t's x (M[i] == K) when no launch in between (nor u's other matrices) writes any byte of x.  One
// image per producing task: the first consumer fixes the matrix; consumers of the same (u, i) share the
// image, a consumer of another matrix of u builds its own with k_prep9_x.  Only tasks whose N takes the GEMM
// path get an image (N > gemv_max_tokens(K)).
// The links alone (no device): prod[t] = the producing task or -1, share[t] = the earlier consumer whose image
// t reads or -1 (t owns an image when it takes the GEMM path), out_mat[u] = the matrix whose y u's epilogue
// turns into an image or -1; gemm[t] = whether t can take the GEMM path at N (N > gemv_max_tokens(K)).
void chain_links(int n, const ggml_hip_chain_task *tasks, int64_t N, int *prod, int *share, int *out_mat, char *gemm) {
    for (int t = 0; t < n; t++) prod[t] = share[t] = out_mat[t] = -1;
    std::vector<int> first_consumer(n, -1);
    for (int t = 0; t < n; t++) {
        const ggml_hip_chain_task &k = tasks[t];
        gemm[t] = N > ghip::gemv_max_tokens(k.K);
        if (!gemm[t]) continue;
        const uint64_t xb = 4 * (uint64_t)k.K * (uint64_t)N;
        int pu = -1, pi = -1;
        for (int u = t - 1; u >= 0; u--) {
            const ggml_hip_chain_task &p = tasks[u];
            int hit = -1;
            bool clash = false;
            for (int i = 0; i < p.nmat; i++) {
                if (p.y[i] == k.x && p.M[i] == k.K) hit = i;
                else if (overlaps(p.y[i], 4 * (uint64_t)p.M[i] * (uint64_t)N, k.x, xb)) clash = true;
            }
            if (hit >= 0 && !clash) pu = u, pi = hit;
            if (hit >= 0 || clash) break;
        }
        if (pu < 0 || !gemm[pu]) continue;            // a GEMV producer has no epilogue image
        if (out_mat[pu] < 0) {                     // the first consumer fixes the producer's image
            out_mat[pu] = pi;
            first_consumer[pu] = t;
            prod[t] = pu;
        } else if (out_mat[pu] == pi) {            // the same (u, i): share the first consumer's image
            prod[t] = pu;
            share[t] = first_consumer[pu];
        }
    }
}

int chain_plan_images(ggml_hip_chain *c) {
    const int n = (int)c->tasks.size();
    std::vector<int> share(n);
    std::vector<char> gemm(n);
    c->prod_task.assign(n, -1);
    c->out_mat.assign(n, -1);
    c->ximg.assign(n, nullptr);
    c->out_img.assign(n, nullptr);
    chain_links(n, c->tasks.data(), c->N, c->prod_task.data(), share.data(), c->out_mat.data(), gemm.data());
    for (int t = 0; t < n; t++) {
        if (!gemm[t]) continue;
        if (share[t] >= 0) {
            c->ximg[t] = c->ximg[share[t]];
            continue;
        }
        void *p = nullptr;
        if (hipMalloc(&p, ghip::gemm9_x_bytes(c->tasks[t].K, c->N)) != hipSuccess) {
            (void)hipGetLastError();
            return fail(GGML_HIP_ERR_NOMEM, "chain x image allocation failed");
        }
        c->owned.push_back(p);
        c->ximg[t] = p;
        if (c->prod_task[t] >= 0) c->out_img[c->prod_task[t]] = p;
    }
    return GGML_HIP_OK;
}

int chain_create(int ntasks, const ggml_hip_chain_task *tasks, int64_t N, ggml_hip_chain **out) {
    ensure_init();
    if (!out) return fail(GGML_HIP_ERR_INVALID, "null out");
    *out = nullptr;
    if (g_device_count == 0) return fail(GGML_HIP_ERR_DEVICE, "no HIP device");
    if (ntasks < 1 || !tasks) return fail(GGML_HIP_ERR_INVALID, "ntasks must be >= 1");
    if (N < 1 || N > ((int64_t)1 << 24)) return fail(GGML_HIP_ERR_INVALID, "N must be 1 .. 2^24");
    for (int t = 0; t < ntasks; t++) {
        const ggml_hip_chain_task &k = tasks[t];
        if (k.nmat < 1 || k.nmat > ghip::GEMV_MULTI_MAX) return fail(GGML_HIP_ERR_INVALID, "nmat must be 1..4");
        if (k.K <= 0 || k.K % 64 != 0 || !k.x || !aligned(k.x, 16))
            return fail(GGML_HIP_ERR_INVALID, "bad x or K (K % 64 == 0, 16-byte aligned x)");
        for (int i = 0; i < k.nmat; i++) {
            if (!k.W[i] || !k.y[i] || k.M[i] <= 0 || !aligned(k.W[i], 16) || !aligned(k.y[i], 4))
                return fail(GGML_HIP_ERR_INVALID, "null / misaligned W or y, or M <= 0");
            // a task's y may not overlap its own x (its rows read x while others write y)
            if (overlaps(k.y[i], 4 * (uint64_t)k.M[i] * (uint64_t)N, k.x, 4 * (uint64_t)k.K * (uint64_t)N))
                return fail(GGML_HIP_ERR_INVALID, "a task's y overlaps its own x");
        }
    }
    auto *c = new ggml_hip_chain();
    c->device = current_device();
    c->N = N;
    c->tasks.assign(tasks, tasks + ntasks);
    if (N > 1) {
        const int rc = chain_plan_images(c);
        if (rc != GGML_HIP_OK) {
            chain_free_images(c);
            delete c;
            return rc;
        }
    }
    if (engine_env() == 1 && N == 1) {
        c->eng_mode = 1;
        (void)chain_engine_on(c);           // a declined chain keeps the per-launch path
    }
    *out = c;
    return GGML_HIP_OK;
}

// One task of an N-token chain: ONE k_gemm9 launch on its x image when ggml_hip_mul_mat_q4_0_multi would run
// it as one (g9_images), the image from the producer's epilogue when the producer ran on k_gemm9 in this pass
// (else k_prep9_x), and this launch's epilogue writing the images its consumers read; otherwise the plain
// sibling call.  Either way y is bitwise ggml_hip_mul_mat_q4_0_multi's.
// GGML_HIP_CHAIN_X9=1 / ggml_hip_debug_set_chain_x9(1): the producers' epilogues write the consumers' x images.
// Off by default: bitwise the same y, but measured 0.7-2.6 % slower over the bench's 4-layer chain
// (profiles/r06_prefill_chain_ab.txt): the image conversion at the end of every tile runs with the tile's
// workgroup alone on its CU (one 154 KB workgroup per CU), +1.3-5 us per launch, while k_prep9_x spreads the
// same work over the whole GPU in ~5 us.
std::atomic<int> g_chain_x9{-1};
bool chain_x9_on() {
    int v = g_chain_x9.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (getenv("GGML_HIP_CHAIN_X9") && atoi(getenv("GGML_HIP_CHAIN_X9")) == 1) ? 1 : 0;
        g_chain_x9.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

int chain_task_n(ggml_hip_chain *c, int t, std::vector<char> &ran9, hipStream_t s) {
    const ggml_hip_chain_task &k = c->tasks[t];
    const void *img[4];
    if (c->ximg[t] && g9_images(k.nmat, k.W, k.M, k.K, c->N, img)) {
        const bool fold = chain_x9_on();
        const int u = c->prod_task[t];
        if (!(fold && u >= 0 && ran9[u] == 2)) HIP_RET(ghip::gemm9_prep_x(k.x, k.K, c->N, c->ximg[t], s));
        uint8_t *xo[4] = {nullptr, nullptr, nullptr, nullptr};
        int64_t ldy[4];
        for (int i = 0; i < k.nmat; i++) ldy[i] = k.M[i];
        // ran9: 2 = this launch's epilogue wrote its consumers' image, 1 = k_gemm9 without it (they prep their own)
        const bool wr = fold && c->out_img[t] && ghip::gemm9_xo_ok(k.M[c->out_mat[t]], c->N);
        if (wr) xo[c->out_mat[t]] = (uint8_t *)c->out_img[t];
        HIP_RET(ghip::gemm9_run_multi(k.nmat, img, k.M, k.K, c->ximg[t], c->N, (float *const *)k.y, ldy, s, xo));
        ran9[t] = wr ? 2 : 1;
        return GGML_HIP_OK;
    }
    ran9[t] = 0;
    return ggml_hip_mul_mat_q4_0_multi(k.nmat, k.W, k.M, k.K, k.x, c->N, (float *const *)k.y, s);
}
}  // namespace

extern "C" {

int ggml_hip_chain_create(int ntasks, const ggml_hip_chain_task *tasks, ggml_hip_chain **out) {
    return chain_create(ntasks, tasks, 1, out);
}

int ggml_hip_chain_create_n(int ntasks, const ggml_hip_chain_task *tasks, int64_t N, ggml_hip_chain **out) {
    return chain_create(ntasks, tasks, N, out);
}

int ggml_hip_debug_chain_links(int ntasks, const ggml_hip_chain_task *tasks, int64_t N, int *prod, int *share) {
    if (ntasks < 1 || !tasks || !prod || !share || N < 1) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    for (int t = 0; t < ntasks; t++)
        if (tasks[t].nmat < 1 || tasks[t].nmat > ghip::GEMV_MULTI_MAX) return fail(GGML_HIP_ERR_INVALID, "nmat must be 1..4");
    std::vector<int> out_mat(ntasks);
    std::vector<char> gemm(ntasks);
    chain_links(ntasks, tasks, N, prod, share, out_mat.data(), gemm.data());
    return GGML_HIP_OK;
}

int ggml_hip_debug_set_chain_x9(int on) {
    if (on < -1 || on > 1) return fail(GGML_HIP_ERR_INVALID, "mode must be -1, 0 or 1");
    g_chain_x9.store(on, std::memory_order_relaxed);          // -1: re-read GGML_HIP_CHAIN_X9
    return GGML_HIP_OK;
}

int ggml_hip_chain_set_engine(ggml_hip_chain *c, int mode) {
    ensure_init();
    if (!c || mode < -1 || mode > 1) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    if (mode == -1) return c->eng ? 1 : 0;
    if (current_device() != c->device) return fail(GGML_HIP_ERR_INVALID, "chain belongs to another device");
    c->eng_mode = mode;
    if (mode == 0) {
        if (c->eng) {
            HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());   // no launch of the plan in flight
            ghip::engine_plan_destroy(c->eng);
            c->eng = nullptr;
        }
        return 0;
    }
    if (chain_engine_on(c)) return 1;
    g_last_error = c->eng_why;
    return 0;
}

// diagnostics (not in the header): per-CU stamps of the engine's last launch (tools/engine_stamps.py)
int ggml_hip_debug_engine_stamps(ggml_hip_chain *c, uint64_t *out, int64_t n) {
    if (!c || !c->eng) return -1;
    (void)GHIP_SYNC(hipDeviceSynchronize)();
    return ghip::engine_stamps(c->eng, out, n);
}

int ggml_hip_chain_engine_info(ggml_hip_chain *c, int64_t *info, int n) {
    if (!c || !info || n < 1) return fail(GGML_HIP_ERR_INVALID, "bad arguments");
    int64_t v[6] = {c->eng ? 1 : 0, 0, 0, 0, 0, 0};
    if (c->eng) ghip::engine_plan_info(c->eng, v + 1);
    for (size_t t = 0; t < c->prod_task.size(); t++) v[5] += c->prod_task[t] >= 0;
    for (int i = 0; i < n && i < 6; i++) info[i] = v[i];
    if (!c->eng && !c->eng_why.empty()) g_last_error = c->eng_why;
    return GGML_HIP_OK;
}

int ggml_hip_chain_launch(ggml_hip_chain *c, void *stream) {
    ensure_init();
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null chain");
    if (current_device() != c->device) return fail(GGML_HIP_ERR_INVALID, "chain belongs to another device");
    hipStream_t s = resolve_stream(stream);
    if (c->eng && !exact_mode()) {          // exact mode: the per-launch exact kernels
        HIP_RET(ghip::engine_launch(c->eng, s));
        return GGML_HIP_OK;
    }
    if (c->N > 1) {
        std::vector<char> ran9(c->tasks.size(), 0);
        for (int t = 0; t < (int)c->tasks.size(); t++) {
            const int rc = chain_task_n(c, t, ran9, s);
            if (rc != GGML_HIP_OK) return rc;
        }
        return GGML_HIP_OK;
    }
    for (const auto &k : c->tasks) {
        const int rc = ggml_hip_mul_mat_q4_0_multi(k.nmat, k.W, k.M, k.K, k.x, 1, (float *const *)k.y, s);
        if (rc != GGML_HIP_OK) return rc;
    }
    return GGML_HIP_OK;
}

int ggml_hip_chain_status(ggml_hip_chain *c) {
    if (!c) return fail(GGML_HIP_ERR_INVALID, "null chain");
    HIP_RET(GHIP_SYNC(hipDeviceSynchronize)());
    if (c->eng) {                           // sticky error bits of the engine's bounded waits
        uint64_t detail = 0;
        const int bits = ghip::engine_status(c->eng, &detail);
        if (bits < 0) return fail(GGML_HIP_ERR_DEVICE, "engine status read failed");
        if (bits) {
            g_last_error = "decode engine: a bounded wait expired (bits " + std::to_string(bits) + ", first at CU " +
                           std::to_string(detail >> 8) + " code " + std::to_string(detail & 0xFF) + ")";
            return bits;
        }
    }
    return 0;
}

int ggml_hip_chain_destroy(ggml_hip_chain *c) {
    if (c && (c->eng || !c->owned.empty())) {
        (void)GHIP_SYNC(hipDeviceSynchronize)();
        if (c->eng) ghip::engine_plan_destroy(c->eng);
        chain_free_images(c);
    }
    delete c;
    return GGML_HIP_OK;
}

}  // extern "C"

extern "C" {

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

}  // extern "C"

extern "C" {

const char *ggml_hip_version(void) { return "ggml-hip q4_0 gfx950 r1"; }

}  // extern "C"
