/*
 * ref_bench.c — TEST INFRASTRUCTURE ONLY: times the REFERENCE ggml CPU path (ggml.c compiled
 * from /root/reference into oracle/_ref by oracle/Makefile) for bench.py's cpu_baseline.
 *
 * One "layer" = the 7 q4_0 mul_mats of a LLaMA-7B decoder layer, ggml_mul_mat nodes.  ref_stack_run
 * puts the mul_mats of all n_layers layer copies into ONE graph and runs one ggml_graph_compute with
 * n_threads worker threads, as llama.cpp runs one graph per token (threads spawned once per graph
 * compute, ggml.c:17540-17571; INIT q8_0 on one thread, COMPUTE row split, ggml.c:11226-11411).
 * ref_layer_run (one graph per mul_mat) is kept for comparison: its per-call thread spawn adds
 * ~0.5 ms per mul_mat.
 * The weights are filled with a repeating pattern of valid q4_0 blocks: the timing does not
 * depend on the values.
 */
#define _POSIX_C_SOURCE 199309L
#include "ggml.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

struct ref_layer {
    struct ggml_context *ctx;
    struct ggml_tensor *out[7];
};

static const int K_[7] = {4096, 4096, 4096, 4096, 4096, 4096, 11008};
static const int M_[7] = {4096, 4096, 4096, 4096, 11008, 11008, 4096};

/* allocate n_layers independent layers (distinct weight memory, > LLC) for N tokens */
void *ref_layers_create(int n_layers, int N) {
    struct ref_layer *L = calloc((size_t)n_layers, sizeof *L);
    for (int l = 0; l < n_layers; l++) {
        size_t need = 64u << 20;
        for (int i = 0; i < 7; i++) need += (size_t)M_[i] * K_[i] / 32 * 18 + (size_t)K_[i] * N * 4 + (size_t)M_[i] * N * 4 + 4096;
        struct ggml_init_params ip = {need, NULL, false};
        L[l].ctx = ggml_init(ip);
        for (int i = 0; i < 7; i++) {
            struct ggml_tensor *w = ggml_new_tensor_2d(L[l].ctx, GGML_TYPE_Q4_0, K_[i], M_[i]);
            struct ggml_tensor *x = ggml_new_tensor_2d(L[l].ctx, GGML_TYPE_F32, K_[i], N);
            uint8_t *wb = (uint8_t *)w->data;
            const size_t nbytes = ggml_nbytes(w);
            for (size_t b = 0; b < nbytes / 18; b++) {          /* d = 0.0125 (fp16 0x2A66), nibbles varied */
                wb[18 * b] = 0x66; wb[18 * b + 1] = 0x2A;
                for (int j = 0; j < 16; j++) wb[18 * b + 2 + j] = (uint8_t)((b * 7 + j * 13 + l) & 0xFF);
            }
            float *xf = (float *)x->data;
            for (int64_t j = 0; j < (int64_t)K_[i] * N; j++) xf[j] = (float)((j * 2654435761u) % 2001) / 1000.0f - 1.0f;
            L[l].out[i] = ggml_mul_mat(L[l].ctx, w, x);
        }
    }
    return L;
}

/* run layer l once with n_threads; returns elapsed seconds */
double ref_layer_run(void *h, int l, int n_threads) {
    struct ref_layer *L = (struct ref_layer *)h;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < 7; i++) {
        struct ggml_cgraph gf = ggml_build_forward(L[l].out[i]);
        gf.n_threads = n_threads;
        ggml_graph_compute(L[l].ctx, &gf);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* all n_layers layers (7 x n_layers mul_mat nodes) in one graph, one ggml_graph_compute; seconds */
double ref_stack_run(void *h, int n_layers, int n_threads) {
    struct ref_layer *L = (struct ref_layer *)h;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    struct ggml_cgraph gf = ggml_build_forward(L[0].out[0]);
    for (int l = 0; l < n_layers; l++)
        for (int i = 0; i < 7; i++) ggml_build_forward_expand(&gf, L[l].out[i]);
    gf.n_threads = n_threads;
    ggml_graph_compute(L[0].ctx, &gf);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

void ref_layers_destroy(void *h, int n_layers) {
    struct ref_layer *L = (struct ref_layer *)h;
    for (int l = 0; l < n_layers; l++) ggml_free(L[l].ctx);
    free(L);
}

/* BASELINE config 1: tests/test-quantize-perf.cpp --type q4_0 --op vec_dot_q --size 16777216 (one
 * 4096 x 4096-value dot on one thread, test-quantize-perf.cpp:339-349; data 0.1 + 2 cos(i + offset),
 * :64-68).  The second operand is quantized with quantize_row_q_dot (q8_0, what the dot reads;
 * test-quantize-perf hands it a q4_0 buffer, which times the same loop).  Per-call seconds of `reps`
 * timed calls after 5 warm-up calls (the test's WARMUP) go to sec[]; returns the dot value. */
float ref_vec_dot_bench(int size, int reps, double *sec) {
    float *a = malloc((size_t)size * 4), *b = malloc((size_t)size * 4);
    void *qa = aligned_alloc(64, ((size_t)size / 32 * 18 + 63) / 64 * 64);
    void *qb = aligned_alloc(64, ((size_t)size / 32 * 34 + 63) / 64 * 64);
    for (int i = 0; i < size; i++) {
        a[i] = 0.1f + 2 * cosf((float)i + 0.0f);
        b[i] = 0.1f + 2 * cosf((float)i + 1.0f);
    }
    struct ggml_init_params ip = {1024, NULL, true};       /* fp16 tables (ggml_init) */
    struct ggml_context *ctx = ggml_init(ip);
    const quantize_fns_t f = ggml_internal_get_quantize_fn(GGML_TYPE_Q4_0);
    f.quantize_row_q(a, qa, size);
    f.quantize_row_q_dot(b, qb, size);
    float r = 0.0f;
    for (int i = 0; i < 5; i++) f.vec_dot_q(size, &r, qa, qb);
    for (int i = 0; i < reps; i++) {
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        f.vec_dot_q(size, &r, qa, qb);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        sec[i] = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    }
    ggml_free(ctx);
    free(a);
    free(b);
    free(qa);
    free(qb);
    return r;
}
