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
#include <string.h>

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
