// ggml-hip-ops.cpp — the non-Q4_0 device ops of a LLaMA layer on the hook path (full offload, SURVEY.md 8f
// row 4): host-built lookup tables of ggml's CPU ops and one launch per ggml node (ggml_ops.hip).
#include "ggml-hip-internal.h"

using namespace ghh;

namespace ghh {

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

std::mutex g_tab_mu;
OpTables g_tabs[GGML_HIP_MAX_DEVICES];
// direct evaluation of the tables' values in the kernels (q4_0_device.h lut_silu / lut_exp) where the device
// reproduces every finite entry bit for bit; GGML_HIP_LUT_DIRECT=0 or ggml_hip_debug_set_lut_direct(0) keeps
// the gathers
std::atomic<int> g_lut_direct{-1};
bool lut_direct_enabled() {
    int v = g_lut_direct.load(std::memory_order_relaxed);
    if (v < 0) {
        v = (!getenv("GGML_HIP_LUT_DIRECT") || atoi(getenv("GGML_HIP_LUT_DIRECT")) != 0) ? 1 : 0;
        g_lut_direct.store(v, std::memory_order_relaxed);
    }
    return v == 1;
}
// the pointers the kernels get: the tables, tagged with bit 0 when they may evaluate directly
void lut_apply(OpTables &t) {
    auto tag = [](uint16_t *p, bool on) { return (uint16_t *)((uintptr_t)p | (on ? 1u : 0u)); };
    const bool on = lut_direct_enabled();
    t.silu = tag(t.silu_raw, on && t.silu_bad == 0);
    t.exp = tag(t.exp_raw, on && t.exp_bad == 0);
}

// ggml_init builds them as fp16(silu(f)) and fp16(expf(f)) for every fp16 bit pattern f with the
// host libm (ggml.c:4246-4254); the same formula with the same libm gives the same 2 x 64 K entries
const OpTables &op_tables(int id, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    OpTables &t = g_tabs[id];
    if (!t.silu_raw) {
        std::vector<uint16_t> silu(65536), ex(65536);
#pragma clang loop vectorize(disable)
        for (int i = 0; i < 65536; i++) {
            const float f = f16_bits_to_f32((uint16_t)i);
            silu[i] = f32_to_f16_bits(f / (1.0f + expf(-f)));
            ex[i] = f32_to_f16_bits(expf(f));
        }
        HIP_FATAL(hipMalloc(&t.silu_raw, 2 * 65536 * sizeof(uint16_t) + 2 * sizeof(int)));
        t.exp_raw = t.silu_raw + 65536;
        int *bad = (int *)(t.exp_raw + 65536);
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(t.silu_raw, silu.data(), 65536 * 2, hipMemcpyHostToDevice, s));
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(t.exp_raw, ex.data(), 65536 * 2, hipMemcpyHostToDevice, s));
        HIP_FATAL(GHIP_SYNC(hipMemsetAsync)(bad, 0, 2 * sizeof(int), s));
        // the kernels' direct evaluation against every finite entry, once per device
        HIP_FATAL(ghip::op_lut_check(t.silu_raw, t.exp_raw, bad, s));
        int hb[2] = {-1, -1};
        HIP_FATAL(GHIP_SYNC(hipMemcpyAsync)(hb, bad, sizeof hb, hipMemcpyDeviceToHost, s));
        HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
        t.silu_bad = hb[0];
        t.exp_bad = hb[1];
        if ((hb[0] || hb[1]) && getenv("GGML_HIP_VERBOSE"))
            fprintf(stderr, "ggml-hip: direct silu / exp differ from the host tables at %d / %d inputs: gathers kept\n",
                    hb[0], hb[1]);
    }
    lut_apply(t);
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


std::atomic<int64_t> g_op_count[gabi::OP_COUNT];      // device nodes run, per ggml op (debug stats)
std::atomic<int64_t> g_host_ns{0};                     // host time inside the taken nodes (debug stats)
std::atomic<int64_t> g_op_ns[gabi::OP_COUNT];          // the same, per op of the node that arrived
// fused launches by chain: add/rms_norm/mul, scale/mask/soft_max, silu/mul, rope/cpy, KQV/merge cpy,
// q4_0 mul_mat run under a pending silu, sibling q4_0 GEMVs (wq|wk|wv, w1|w3) run as one group,
// independent rope / rope->cpy / cpy nodes held behind a group run as one launch, the decode
// soft_max chain with its KQV and merged copy as one launch, the decode norm / silu chains in the GEMV
// prologue (9, 10), the prefill chains that wrote the k_gemm9 x image of their output (11), the decode
// q|k|v GEMVs that ran the held rope / copy nodes in their epilogue (12), the decode w1|w3 GEMVs that ran
// silu -> mul in theirs (13), the decode soft_max -> KQV launches that computed KQ too (14)
std::atomic<int64_t> g_fused[N_FUSED];

// fused_cpy: a CPY node consuming t (rope -> cpy into the K cache; f16 mul_mat -> permute(0,2,1,3)
// -> contiguous cpy), checked by try_fuse; its destination is written by t's own kernel
void run_device_op(tensor *t, const tensor *fused_cpy) {
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

}  // namespace ghh

extern "C" {

// not in the public header: the fp16-table ops' direct evaluation (out[0] silu mode, [1] silu mismatches of the
// device check, [2] exp mode, [3] exp mismatches; mode 1 = direct, 0 = table gathers); on: 1 / 0 sets the
// switch, -1 only reads (device 0's tables, built on first use)
int ggml_hip_debug_lut_direct(int on, int *out) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    flush_deferred();
    if (on >= 0) g_lut_direct.store(on ? 1 : 0, std::memory_order_relaxed);
    HIP_FATAL(hipSetDevice(g_main_device));
    const OpTables &t = op_tables(g_main_device, g_dev[g_main_device].stream);
    if (out) {
        out[0] = ((uintptr_t)t.silu & 1) ? 1 : 0;
        out[1] = t.silu_bad;
        out[2] = ((uintptr_t)t.exp & 1) ? 1 : 0;
        out[3] = t.exp_bad;
    }
    return GGML_HIP_OK;
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

}  // extern "C"

extern "C" {

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

// debug: the decode sibling GEMV with its x prologue (kind 0 plain x = b, 1 [a +] b -> rms_norm -> * w, 2 silu(a)
// * b) and optionally an epilogue (epi: a ghip::GemvEpi, its table filled here for glu), on device pointers.
// reps > 0: the launch is repeated reps times between two events and *us receives the mean (tools/gemv_epi_ab.py);
// the outputs are those of the last launch.
int ggml_hip_debug_gemv_norm(int nmat, const void *const *W, const int64_t *M, int64_t K, int kind, const float *a,
                             const float *b, const float *w, float *sum, float *norm, float *out, float *const *y,
                             const void *epi, int reps, float *us) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    if (nmat < 1 || nmat > 4 || kind < 0 || kind > 2) return fail(GGML_HIP_ERR_INVALID, "bad gemv_norm case");
    flush_deferred();
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    hipStream_t s = g_dev[id].stream;
    const OpTables &tb = op_tables(id, s);
    ghip::GemvEpi ep{};
    if (epi) {
        memcpy(&ep, epi, sizeof ep);
        if (ep.glu) ep.table = tb.silu;
    }
    int64_t ldy[4];
    for (int i = 0; i < nmat; i++) ldy[i] = M[i];
    const ghip::GemvNorm nrm{a, w, sum, norm, out, kind, kind == 2 ? tb.silu : nullptr};
    auto run = [&]() -> hipError_t {
        if (kind == 0) return ghip::gemv_q4_0_multi(nmat, W, M, K, b, 1, y, ldy, g_dev[id].info, s);
        return ghip::gemv_q4_0_multi_norm(nmat, W, M, K, b, nrm, y, ldy, g_dev[id].info, s, epi ? &ep : nullptr);
    };
    HIP_RET(run());
    if (reps > 0) {
        hipEvent_t e0, e1;
        HIP_FATAL(GHIP_SYNC(hipEventCreate)(&e0));
        HIP_FATAL(GHIP_SYNC(hipEventCreate)(&e1));
        HIP_FATAL(GHIP_SYNC(hipEventRecord)(e0, s));
        for (int r = 0; r < reps; r++) HIP_RET(run());
        HIP_FATAL(GHIP_SYNC(hipEventRecord)(e1, s));
        HIP_FATAL(GHIP_SYNC(hipEventSynchronize)(e1));
        float ms = 0.0f;
        HIP_FATAL(hipEventElapsedTime(&ms, e0, e1));
        if (us) *us = 1000.0f * ms / (float)reps;
        HIP_FATAL(hipEventDestroy(e0));
        HIP_FATAL(hipEventDestroy(e1));
    }
    HIP_FATAL(GHIP_SYNC(hipStreamSynchronize)(s));
    return GGML_HIP_OK;
}

// debug: the decode attention of one query row per head on device pointers: fused = 1 the one launch
// (op_kq_softmax_kqv), 0 KQ's own launch (op_mul_mat_f16_f32) then op_softmax_kqv; kq receives KQ (fused = 0) or
// the softmax row (both: sm), kqv the [nhead][nout] output.  reps > 0: timed as ggml_hip_debug_gemv_norm.
int ggml_hip_debug_attn_decode(int fused, const void *ks, int64_t nb01k, int64_t nb02k, const float *q, int64_t nb02q,
                               int hd, const void *vs, int64_t nb01v, int64_t nb02v, int64_t nkv, int64_t nhead,
                               int64_t nout, int n_past, float scale, float *kq, float *sm, float *kqv, int reps, float *us) {
    ensure_init();
    if (g_device_count == 0) return GGML_HIP_ERR_UNSUPPORTED;
    flush_deferred();
    const int id = g_main_device;
    HIP_FATAL(hipSetDevice(id));
    hipStream_t s = g_dev[id].stream;
    const OpTables &tb = op_tables(id, s);
    auto run = [&]() -> hipError_t {
        if (fused)
            return ghip::op_kq_softmax_kqv(ks, nb01k, nb02k, q, nb02q, hd, nullptr, nullptr, nullptr, sm, scale, n_past,
                                           tb.exp, nkv, nhead, vs, nb01v, nb02v, nout, kqv, nullptr, s);
        hipError_t e = ghip::op_mul_mat_f16_f32(ks, q, kq, hd, nkv, 1, nhead, nb01k, nb02k, nb02q, nb02q, s, nullptr,
                                                 exact_mode() ? -1 : -2);
        if (e != hipSuccess) return e;
        return ghip::op_softmax_kqv(kq, nullptr, nullptr, sm, scale, n_past, tb.exp, nkv, nhead, vs, nb01v, nb02v, nout,
                                    kqv, nullptr, s);
    };
    HIP_RET(run());
    if (reps > 0) {
        hipEvent_t e0, e1;
        HIP_FATAL(GHIP_SYNC(hipEventCreate)(&e0));
        HIP_FATAL(GHIP_SYNC(hipEventCreate)(&e1));
        HIP_FATAL(GHIP_SYNC(hipEventRecord)(e0, s));
        for (int r = 0; r < reps; r++) HIP_RET(run());
        HIP_FATAL(GHIP_SYNC(hipEventRecord)(e1, s));
        HIP_FATAL(GHIP_SYNC(hipEventSynchronize)(e1));
        float ms = 0.0f;
        HIP_FATAL(hipEventElapsedTime(&ms, e0, e1));
        if (us) *us = 1000.0f * ms / (float)reps;
        HIP_FATAL(hipEventDestroy(e0));
        HIP_FATAL(hipEventDestroy(e1));
    }
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

}  // extern "C"
