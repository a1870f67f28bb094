// ggml-hip-tensor.cpp — the ggml tensor ABI (ggml-cuda.h:15-36 restated as ggml_hip_*): buffers of graph
// tensors, transform_tensor / free_data, the q4_0 mul_mat of a node and ggml_hip_compute_forward.
#include "ggml-hip-internal.h"

using namespace ghh;

namespace ghh {

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

}  // namespace ghh

namespace ghh {

// host copies made by ggml_hip_transform_tensor for tensors that stay on the CPU
std::mutex g_host_copy_mu;
std::unordered_map<const void *, void *> g_host_copies;

}  // namespace ghh

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

namespace ghh {

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
    const uint64_t call_id = wcache_next_call_id();
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
                    wcache_note_image(id, w, image_format() == 9 ? ghip::gemm9_w_bytes(K, rows) : ghip::gemm8_w_bytes(K, rows),
                                      call_id);
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

}  // namespace ghh

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
    if (!hook_holding()) {
        snap_reset();                      // nothing held: the copies are garbage
    } else if (hook_seen(t)) {
        flush_deferred();                  // t arrives again: a new graph at the old addresses
    }
    // with the recorder on, the node's launches on the main stream are recorded (launch.h): mode 1 submits
    // them as HIP graphs when the node returns; mode 2's launcher thread issues them on its own, so the ring
    // stays open across nodes (the main thread never waits for it between nodes: every entry point and
    // every other HIP call of the backend drains it first, GHIP_SYNC / flush_deferred)
    g_eval_computed = true;
    const int gmode = graph_enabled() ? graph_apply_mode() : 0;
    ghip::rec_enable(g_dev[g_main_device].stream, gmode != 0);
    execute_node(t);
    if (gmode == 1) ghip::rec_enable(g_dev[g_main_device].stream, false);
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

}  // extern "C"
