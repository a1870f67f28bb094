/*
 * gen_golden.c — generates the golden fixtures in tests/golden/ from the
 * REFERENCE ggml CPU path, compiled out of tree from /root/reference/ggml.c by
 * oracle/Makefile (target `golden`).  Built twice:
 *   gen_golden_avx2   : ggml.c with -march=x86-64-v3 -> AVX2 branches
 *                       (quantize_row_q8_0 ggml.c:1192-1275, vec_dot ggml.c:2412-2435)
 *   gen_golden_scalar : ggml.c with -march=x86-64   -> scalar branches
 *                       (ggml.c:1276-1279, ggml.c:2588-2606)
 * Each run writes <variant>_*.bin plus a JSON manifest fragment.  Inputs come
 * from the repo's splitmix64 + Box-Muller generator (oracle_fill_gaussian) so
 * they are reproducible without the reference.
 *
 * Usage: gen_golden_<variant> <outdir> <variant>
 */
#include "ggml.h"
#include "q4_0_oracle.h"   /* only for oracle_fill_gaussian (input synthesis) */

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const char *g_out;
static const char *g_var;
static FILE *g_manifest;
static int g_first = 1;

static void dump(const char *name, const void *p, size_t n, const char *dtype, const char *shape) {
    char path[1024];
    snprintf(path, sizeof path, "%s/%s_%s.bin", g_out, g_var, name);
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(p, 1, n, f) != n) { perror(path); exit(1); }
    fclose(f);
    fprintf(g_manifest, "%s    \"%s_%s\": {\"file\": \"%s_%s.bin\", \"bytes\": %zu, \"dtype\": \"%s\", \"shape\": %s}",
            g_first ? "" : ",\n", g_var, name, g_var, name, n, dtype, shape);
    g_first = 0;
}

/* y[N][M] = ggml_mul_mat(W[M][K] q4_0, x[N][K] f32) through the real graph
 * executor (ggml.c:5950 ctor, 17165 graph_compute, 11226 mul_mat_q_f32). */
static void ref_mul_mat(const void *wq, int K, int M, const float *x, int N, float *y, int nthreads) {
    const size_t need = (size_t)M * K + (size_t)N * K * 4 + (size_t)N * M * 4 + (64u << 20);
    struct ggml_init_params ip = {need, NULL, false};
    struct ggml_context *ctx = ggml_init(ip);
    struct ggml_tensor *w = ggml_new_tensor_2d(ctx, GGML_TYPE_Q4_0, K, M);
    struct ggml_tensor *xt = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
    memcpy(w->data, wq, ggml_nbytes(w));
    memcpy(xt->data, x, ggml_nbytes(xt));
    struct ggml_tensor *out = ggml_mul_mat(ctx, w, xt);
    struct ggml_cgraph gf = ggml_build_forward(out);
    gf.n_threads = nthreads;
    ggml_graph_compute(ctx, &gf);
    memcpy(y, out->data, (size_t)N * M * 4);
    ggml_free(ctx);
}

int main(int argc, char **argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s outdir variant\n", argv[0]); return 2; }
    g_out = argv[1];
    g_var = argv[2];
    char mpath[1024];
    snprintf(mpath, sizeof mpath, "%s/%s_manifest.json", g_out, g_var);
    g_manifest = fopen(mpath, "w");
    fprintf(g_manifest, "{\n");

    { /* fp16 table init (scalar build looks fp16 up in table_f32_f16) */
        struct ggml_init_params ip = {1 << 20, NULL, false};
        ggml_free(ggml_init(ip));
    }
    quantize_fns_t q4 = ggml_internal_get_quantize_fn(GGML_TYPE_Q4_0);
    quantize_fns_t q8 = ggml_internal_get_quantize_fn(GGML_TYPE_Q8_0);
    char shape[128];

    /* (1)-(4) LLaMA-7B-shaped slice: W 64 x 4096 from N(0,0.02); x 4 x 4096 from N(0,1) */
    {
        const int K = 4096, M = 64, N = 4;
        const int nb = K / 32;
        float *wf = malloc((size_t)M * K * 4);
        float *x = malloc((size_t)N * K * 4);
        oracle_fill_gaussian(wf, (size_t)M * K, 0x5EED0001ull, 0.0f, 0.02f);
        oracle_fill_gaussian(x, (size_t)N * K, 0x5EED0002ull, 0.0f, 1.0f);
        uint8_t *wq = malloc((size_t)M * nb * 18);
        int64_t hist[16] = {0};
        ggml_quantize_q4_0(wf, wq, M * K, K, hist);           /* A3, ggml.c:19157 */
        snprintf(shape, sizeof shape, "[%d, %d]", M, nb * 18);
        dump("w4096_q4_0", wq, (size_t)M * nb * 18, "u8", shape);
        dump("w4096_hist", hist, sizeof hist, "i64", "[16]");
        snprintf(shape, sizeof shape, "[%d, %d]", N, K);
        dump("x4096_f32", x, (size_t)N * K * 4, "f32", shape);

        uint8_t *xq = malloc((size_t)N * nb * 34), *xr = malloc((size_t)N * nb * 34);
        for (int n = 0; n < N; n++) {
            q4.quantize_row_q_dot(x + (size_t)n * K, xq + (size_t)n * nb * 34, K);    /* A5 as mul_mat calls it */
            q8.quantize_row_q_reference(x + (size_t)n * K, xr + (size_t)n * nb * 34, K);
        }
        snprintf(shape, sizeof shape, "[%d, %d]", N, nb * 34);
        dump("x4096_q8_0", xq, (size_t)N * nb * 34, "u8", shape);
        dump("x4096_q8_0_scalarref", xr, (size_t)N * nb * 34, "u8", shape);

        float *y = malloc((size_t)N * M * 4), *yd = malloc((size_t)N * M * 4);
        ref_mul_mat(wq, K, M, x, N, y, 4);
        for (int n = 0; n < N; n++)
            for (int m = 0; m < M; m++)
                q4.vec_dot_q(K, &yd[(size_t)n * M + m], wq + (size_t)m * nb * 18, xq + (size_t)n * nb * 34);
        snprintf(shape, sizeof shape, "[%d, %d]", N, M);
        dump("y4096_mul_mat", y, (size_t)N * M * 4, "f32", shape);
        dump("y4096_vec_dot", yd, (size_t)N * M * 4, "f32", shape);

        float *deq = malloc((size_t)2 * K * 4);
        q4.dequantize_row_q(wq, deq, 2 * K);                    /* A4 on first two rows */
        snprintf(shape, sizeof shape, "[2, %d]", K);
        dump("w4096_dequant_rows01", deq, (size_t)2 * K * 4, "f32", shape);
        free(wf); free(x); free(wq); free(xq); free(xr); free(y); free(yd); free(deq);
    }

    /* (5) q8_0 tie-rounding and scale-edge blocks (K = 32 * 8) */
    {
        const int K = 256, nb = 8;
        float x[256];
        for (int i = 0; i < K; i++) x[i] = 0.0f;
        /* block 0: amax 127 -> id 1 exactly; half-integers expose rint vs roundf */
        const float t0[] = {127.f, 2.5f, -0.5f, 0.5f, 1.5f, -1.5f, -2.5f, 3.5f, 126.5f, -126.5f, 0.25f, -0.75f};
        for (int i = 0; i < 12; i++) x[i] = t0[i];
        /* block 1: amax 63.5 -> id = 2 exactly; x*id lands on .5 for quarter values */
        for (int i = 0; i < 32; i++) x[32 + i] = (i == 0) ? 63.5f : (float)(i - 16) * 0.25f + 0.125f * (i & 1);
        /* block 2: all zero (d = 0, id = 0) */
        /* block 3: tiny amax -> fp16-subnormal d */
        for (int i = 0; i < 32; i++) x[96 + i] = 1e-5f * (float)((i * 7) % 13 - 6) / 6.0f;
        /* block 4: d underflows to fp16 zero while q stays non-zero */
        for (int i = 0; i < 32; i++) x[128 + i] = 1e-8f * (float)((i * 5) % 11 - 5) / 5.0f;
        /* block 5: large values -> d near fp16 max range */
        for (int i = 0; i < 32; i++) x[160 + i] = 60000.0f * (float)((i * 3) % 17 - 8) / 8.0f;
        /* block 6: single non-zero (negative) */
        x[192 + 17] = -3.0f;
        /* block 7: values where 127/amax and 1/(amax/127) round differently */
        for (int i = 0; i < 32; i++) x[224 + i] = 0.37f + 0.0913f * (float)i - 1.1f * (float)(i & 3);
        uint8_t qa[8 * 34], qr[8 * 34];
        q4.quantize_row_q_dot(x, qa, K);
        q8.quantize_row_q_reference(x, qr, K);
        snprintf(shape, sizeof shape, "[%d]", K);
        dump("tie_x_f32", x, sizeof x, "f32", shape);
        snprintf(shape, sizeof shape, "[%d, 34]", nb);
        dump("tie_q8_0", qa, sizeof qa, "u8", shape);
        dump("tie_q8_0_scalarref", qr, sizeof qr, "u8", shape);
    }

    /* (6) Falcon-7B QKV shape slice: K = 4544 (142 blocks, rows only 4-byte aligned) */
    {
        const int K = 4544, M = 8, N = 2, nb = K / 32;
        float *wf = malloc((size_t)M * K * 4), *x = malloc((size_t)N * K * 4);
        oracle_fill_gaussian(wf, (size_t)M * K, 0x5EED0003ull, 0.0f, 0.02f);
        oracle_fill_gaussian(x, (size_t)N * K, 0x5EED0004ull, 0.0f, 1.0f);
        uint8_t *wq = malloc((size_t)M * nb * 18);
        int64_t hist[16] = {0};
        ggml_quantize_q4_0(wf, wq, M * K, K, hist);
        float *y = malloc((size_t)N * M * 4);
        ref_mul_mat(wq, K, M, x, N, y, 3);
        snprintf(shape, sizeof shape, "[%d, %d]", M, nb * 18);
        dump("w4544_q4_0", wq, (size_t)M * nb * 18, "u8", shape);
        snprintf(shape, sizeof shape, "[%d, %d]", N, K);
        dump("x4544_f32", x, (size_t)N * K * 4, "f32", shape);
        snprintf(shape, sizeof shape, "[%d, %d]", N, M);
        dump("y4544_mul_mat", y, (size_t)N * M * 4, "f32", shape);
        free(wf); free(x); free(wq); free(y);
    }

    /* (7) q4_0 quantizer ties: negative max first -> d = +max/8; zero block; equal |v| */
    {
        const int K = 128;
        float w[128];
        for (int i = 0; i < K; i++) w[i] = 0.0f;
        w[0] = -1.0f; w[1] = 1.0f; w[2] = 0.5f; w[3] = -0.0625f; w[4] = 0.9375f;   /* block 0 */
        /* block 1: all zero */
        for (int i = 0; i < 32; i++) w[64 + i] = 0.01f * (float)(i - 16);          /* block 2 */
        w[96] = 2.0f; w[97] = -2.0f; w[98] = 0.125f; w[99] = -1.875f;               /* block 3 */
        uint8_t q[4 * 18];
        int64_t hist[16] = {0};
        ggml_quantize_q4_0(w, q, K, K, hist);
        dump("q4tie_w_f32", w, sizeof w, "f32", "[128]");
        dump("q4tie_q4_0", q, sizeof q, "u8", "[4, 18]");
    }

    /* test-quantize-fns synthetic data (tests/test-quantize-fns.cpp:26-30, n = 4096):
     * quantized bytes + the dot of data vs offset data, for the tolerance tests */
    {
        const int n = 4096, nb = n / 32;
        float *a = malloc(n * 4), *b = malloc(n * 4);
        for (int i = 0; i < n; i++) { a[i] = 0.1f + 2 * cosf((float)i + 0.0f); b[i] = 0.1f + 2 * cosf((float)i + 1.0f); }
        uint8_t *qa = malloc(nb * 18), *qb = malloc(nb * 34);
        q4.quantize_row_q(a, qa, n);
        q4.quantize_row_q_dot(b, qb, n);
        float dot = 0.0f;
        q4.vec_dot_q(n, &dot, qa, qb);
        dump("qfns_a_f32", a, n * 4, "f32", "[4096]");
        dump("qfns_b_f32", b, n * 4, "f32", "[4096]");
        dump("qfns_a_q4_0", qa, nb * 18, "u8", "[128, 18]");
        dump("qfns_b_q8_0", qb, nb * 34, "u8", "[128, 34]");
        dump("qfns_dot", &dot, 4, "f32", "[1]");
        free(a); free(b); free(qa); free(qb);
    }

    fprintf(g_manifest, "\n}\n");
    fclose(g_manifest);
    return 0;
}
