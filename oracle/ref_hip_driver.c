/*
 * ref_hip_driver.c — TEST INFRASTRUCTURE ONLY (the CALLER side of the drop-in, not a checker of
 * numbers): the reference's own ggml.c, compiled with -DGGML_USE_CUBLAS from /root/reference and
 * linked against libggml_hip_cuda.so (include/ggml-hip-cuda-abi.h), runs a q4_0 mul_mat graph.
 * ggml.c's hooks then call into the MI355X backend exactly where they call the CUDA backend:
 * ggml_init -> ggml_init_cublas (ggml.c:4282-4283), the planner's can_mul_mat (17283-17288),
 * ggml_compute_forward -> ggml_cuda_compute_forward (15645-15652).  The weight is offloaded the way
 * llama.cpp's loader does it (backend = GPU, then ggml_cuda_transform_tensor, llama.cpp:670-685).
 */
#include "ggml.h"
#include "ggml-cuda.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* from include/ggml-hip.h (libggml_hip.so, loaded as the shim's dependency) */
int ggml_hip_device_synchronize(void);
int ggml_hip_memcpy_d2h(void *dst, const void *src, size_t size, void *stream);
int ggml_hip_weight_cache_stats(int64_t *hits, int64_t *misses, int64_t *resident_bytes);
int64_t ggml_hip_weight_cache_invalidations(void);

/* y[N][M] = mul_mat(W q4_0 [M][K], x f32 [N][K]) through ggml_graph_compute with n_threads.
 * offload: 0 = weight stays a CPU tensor (ggml decides via can_mul_mat: N >= 32 goes to the GPU
 * with per-call upload, like the reference), 1 = GGML_BACKEND_GPU, 2 = GGML_BACKEND_GPU_SPLIT.
 * Returns the dst tensor's backend after compute (0 CPU) or -1 on error. */
int refhip_mul_mat(const void *wq, int K, int M, const float *x, int N, float *y, int offload, int n_threads) {
    const size_t wbytes = (size_t)M * (K / 32) * 18;
    const size_t need = wbytes + (size_t)K * N * 4 + (size_t)M * N * 4 + (1u << 20);
    struct ggml_init_params ip = {need, NULL, false};
    struct ggml_context *ctx = ggml_init(ip);
    if (!ctx) return -1;
    struct ggml_tensor *w = ggml_new_tensor_2d(ctx, GGML_TYPE_Q4_0, K, M);
    struct ggml_tensor *xt = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
    memcpy(w->data, wq, wbytes);
    memcpy(xt->data, x, (size_t)K * N * 4);
    if (offload) {
        w->backend = offload == 2 ? GGML_BACKEND_GPU_SPLIT : GGML_BACKEND_GPU;
        ggml_cuda_transform_tensor(w->data, w);
    }
    struct ggml_tensor *out = ggml_mul_mat(ctx, w, xt);
    struct ggml_cgraph gf = ggml_build_forward(out);
    gf.n_threads = n_threads;
    ggml_graph_compute(ctx, &gf);
    memcpy(y, out->data, (size_t)M * N * 4);
    const int be = (int)out->backend;
    if (offload) ggml_cuda_free_data(w);
    ggml_free(ctx);
    return be;
}

/* 1 when this ggml.c was built with the GPU backend hooks (ggml.c:19465-19470) */
int refhip_has_gpublas(void) { return ggml_cpu_has_cublas(); }

/* The reference's LoRA apply (llama.cpp:2935-2967) rewrites a Q4_0 weight in place with a ggml graph
 * (ggml_add_inplace(w, BA) -> ggml_compute_forward_add_q_f32).  Here: y_before = W x (N >= 32: the
 * backend takes it and caches the CPU weight), then W += delta by ggml_add_inplace on the CPU, then
 * y_after = W x again through the backend.  wq_after receives the rewritten weight bytes; counts[0..2] =
 * cache hits, misses, invalidations after the last mul_mat.  Returns 0, or -1 on error. */
int refhip_lora_add(const void *wq, int K, int M, const float *x, int N, const float *delta, float *y_before,
                    float *y_after, void *wq_after, int64_t *counts, int n_threads) {
    const size_t wbytes = (size_t)M * (K / 32) * 18;
    const size_t need = wbytes + (size_t)K * N * 4 + (size_t)K * M * 4 + 2 * (size_t)M * N * 4 + (4u << 20);
    struct ggml_init_params ip = {need, NULL, false};
    struct ggml_context *ctx = ggml_init(ip);
    if (!ctx) return -1;
    struct ggml_tensor *w = ggml_new_tensor_2d(ctx, GGML_TYPE_Q4_0, K, M);
    struct ggml_tensor *xt = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
    struct ggml_tensor *dt = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, M);
    memcpy(w->data, wq, wbytes);
    memcpy(xt->data, x, (size_t)K * N * 4);
    memcpy(dt->data, delta, (size_t)K * M * 4);
    struct ggml_tensor *o1 = ggml_mul_mat(ctx, w, xt);
    struct ggml_cgraph g1 = ggml_build_forward(o1);
    g1.n_threads = n_threads;
    ggml_graph_compute(ctx, &g1);
    memcpy(y_before, o1->data, (size_t)M * N * 4);
    struct ggml_tensor *r = ggml_add_inplace(ctx, w, dt);
    struct ggml_cgraph g2 = ggml_build_forward(r);
    g2.n_threads = n_threads;
    ggml_graph_compute(ctx, &g2);
    struct ggml_tensor *o2 = ggml_mul_mat(ctx, w, xt);
    struct ggml_cgraph g3 = ggml_build_forward(o2);
    g3.n_threads = n_threads;
    ggml_graph_compute(ctx, &g3);
    memcpy(y_after, o2->data, (size_t)M * N * 4);
    memcpy(wq_after, w->data, wbytes);
    int64_t resident;
    ggml_hip_weight_cache_stats(&counts[0], &counts[1], &resident);
    counts[2] = ggml_hip_weight_cache_invalidations();
    ggml_free(ctx);
    return 0;
}

/* A graph that ENDS on a device-only node: y = silu(rms_norm(x)) with both nodes offloaded
 * (ggml_cuda_assign_buffers_no_scratch, as llama.cpp offloads graph tensors).  The backend defers the
 * final silu (a launch-fusion candidate), so it is still held when ggml_graph_compute returns; the
 * context is then freed and, with poison, its arena overwritten before the backend is synchronized
 * (which runs the held node).  y receives the device result; y_cpu the same graph on ggml's CPU ops.
 * Returns 0, or -1 on error. */
int refhip_device_tail(const float *x, int n, int rows, float *y, float *y_cpu, int poison, int n_threads) {
    const size_t need = (size_t)n * rows * 4 * 4 + (1u << 20);
    void *mem = malloc(need);
    if (!mem) return -1;
    for (int dev = 1; dev >= 0; dev--) {
        struct ggml_init_params ip = {need, mem, false};
        struct ggml_context *ctx = ggml_init(ip);
        if (!ctx) return -1;
        struct ggml_tensor *xt = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, n, rows);
        memcpy(xt->data, x, (size_t)n * rows * 4);
        struct ggml_tensor *a = ggml_rms_norm(ctx, xt);
        if (dev) ggml_cuda_assign_buffers_no_scratch(a);
        struct ggml_tensor *b = ggml_silu(ctx, a);
        if (dev) ggml_cuda_assign_buffers_no_scratch(b);
        struct ggml_cgraph gf = ggml_build_forward(b);
        gf.n_threads = n_threads;
        ggml_graph_compute(ctx, &gf);
        if (dev) {
            void *d = ((struct ggml_tensor_extra_gpu *)b->extra)->data_device[0];
            ggml_free(ctx);
            if (poison) memset(mem, 0xA5, need);
            if (ggml_hip_device_synchronize() != 0) return -1;
            if (ggml_hip_memcpy_d2h(y, d, (size_t)n * rows * 4, NULL) != 0) return -1;
        } else {
            memcpy(y_cpu, b->data, (size_t)n * rows * 4);
            ggml_free(ctx);
        }
    }
    free(mem);
    return 0;
}
