/*
 * q4_0_oracle.c — CPU restatement of the reference q4_0 x q8_0 mul_mat path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline).  See
 * q4_0_oracle.h for the function -> reference file:line map.  Never linked by
 * the product library.
 *
 * Build: oracle/Makefile (gcc -O3 -std=c11 -ffp-contract=off; the AVX2 SIMD
 * helpers carry their own target attribute so the library still loads on a
 * host without AVX2 and falls back to the portable emulation).
 */
#define _GNU_SOURCE
#include "q4_0_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

/* ------------------------------------------------------------------------ */
/* fp16 <-> fp32.  The reference (x86, -march=native) uses F16C
 * _cvtss_sh(x, 0) = round-to-nearest-even, and _cvtsh_ss (exact), ggml.c:284-300. */

uint16_t oracle_fp32_to_fp16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t a = u & 0x7FFFFFFFu;
    if (a > 0x7F800000u) {                  /* NaN -> quiet NaN, payload kept (vcvtps2ph) */
        return (uint16_t)(sign | 0x7E00u | ((a >> 13) & 0x3FFu));
    }
    if (a >= 0x477FF000u) {                 /* >= 65520 rounds to infinity */
        return (uint16_t)(sign | 0x7C00u);
    }
    if (a >= 0x38800000u) {                 /* normal half */
        const uint32_t e = (a >> 23) - 127u + 15u;
        const uint32_t m = a & 0x7FFFFFu;
        uint32_t h = (e << 10) | (m >> 13);
        const uint32_t rem = m & 0x1FFFu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;   /* carry may reach inf: correct */
        return (uint16_t)(sign | h);
    }
    if (a < 0x33000000u) {                  /* < 2^-25 (incl. exactly 2^-25 tie -> even 0) */
        return (uint16_t)sign;
    }
    /* subnormal half: value / 2^-24 with RNE */
    const uint32_t e = a >> 23;             /* 102..112 */
    const uint32_t m = (a & 0x7FFFFFu) | 0x800000u;
    const uint32_t shift = 126u - e;        /* 14..24 */
    uint32_t k = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1u);
    const uint32_t half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (k & 1u))) k++;
    return (uint16_t)(sign | k);
}

float oracle_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = ((uint32_t)h >> 10) & 0x1Fu;
    uint32_t m = (uint32_t)h & 0x3FFu;
    uint32_t u;
    if (e == 0x1Fu) {
        u = sign | 0x7F800000u | (m << 13);
    } else if (e != 0) {
        u = sign | ((e + 112u) << 23) | (m << 13);
    } else if (m == 0) {
        u = sign;
    } else {                                 /* subnormal: normalise */
        e = 113u;
        while ((m & 0x400u) == 0) { m <<= 1; e--; }
        u = sign | (e << 23) | ((m & 0x3FFu) << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline void wr16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

/* ------------------------------------------------------------------------ */
/* A3: quantize_row_q4_0_reference, ggml.c:918-953.
 * max = the signed value of largest magnitude (first occurrence wins),
 * d = max / -8 (fp32), id = 1/d, q = min(15, (int8)(v*id + 8.5)), d stored fp16. */
void oracle_quantize_row_q4_0(const float *x, void *vy, int k) {
    uint8_t *y = (uint8_t *)vy;
    const int nb = k / ORACLE_QK;
    for (int i = 0; i < nb; i++) {
        const float *xb = x + (size_t)i * ORACLE_QK;
        float amax = 0.0f, vmax = 0.0f;
        for (int j = 0; j < ORACLE_QK; j++) {
            const float v = xb[j];
            if (amax < fabsf(v)) { amax = fabsf(v); vmax = v; }
        }
        const float d = vmax / -8;
        const float id = d ? 1.0f / d : 0.0f;
        uint8_t *blk = y + (size_t)i * ORACLE_Q4_0_BLOCK_BYTES;
        wr16(blk, oracle_fp32_to_fp16(d));
        for (int j = 0; j < ORACLE_QK / 2; j++) {
            const float x0 = xb[j] * id;
            const float x1 = xb[j + ORACLE_QK / 2] * id;
            int q0 = (int8_t)(x0 + 8.5f);
            int q1 = (int8_t)(x1 + 8.5f);
            if (q0 > 15) q0 = 15;
            if (q1 > 15) q1 = 15;
            blk[2 + j] = (uint8_t)((uint8_t)q0 | ((uint8_t)q1 << 4));
        }
    }
}

/* ggml_quantize_q4_0, ggml.c:19157-19178: quantize n floats in rows of k,
 * accumulate the 16-bin nibble histogram, return bytes written. */
size_t oracle_quantize_q4_0(const float *src, void *dst, int n, int k, int64_t *hist) {
    const int nb = k / ORACLE_QK;
    for (int b = 0; b < n; b += k) {
        uint8_t *y = (uint8_t *)dst + (size_t)(b / ORACLE_QK) * ORACLE_Q4_0_BLOCK_BYTES;
        oracle_quantize_row_q4_0(src + b, y, k);
        if (hist) {
            for (int i = 0; i < nb; i++) {
                for (int j = 0; j < ORACLE_QK / 2; j++) {
                    const uint8_t q = y[(size_t)i * ORACLE_Q4_0_BLOCK_BYTES + 2 + j];
                    hist[q & 0x0F]++;
                    hist[q >> 4]++;
                }
            }
        }
    }
    return (size_t)(n / ORACLE_QK) * ORACLE_Q4_0_BLOCK_BYTES;
}

/* A4: dequantize_row_q4_0, ggml.c:1500-1518 */
void oracle_dequantize_row_q4_0(const void *vx, float *y, int k) {
    const uint8_t *x = (const uint8_t *)vx;
    const int nb = k / ORACLE_QK;
    for (int i = 0; i < nb; i++) {
        const uint8_t *blk = x + (size_t)i * ORACLE_Q4_0_BLOCK_BYTES;
        const float d = oracle_fp16_to_fp32(rd16(blk));
        for (int j = 0; j < ORACLE_QK / 2; j++) {
            y[i * ORACLE_QK + j] = (float)((blk[2 + j] & 0x0F) - 8) * d;
            y[i * ORACLE_QK + j + ORACLE_QK / 2] = (float)((blk[2 + j] >> 4) - 8) * d;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* A5: q8_0 activation quantizer. */

/* _mm256_round_ps(.., nearest-even) -> _mm256_cvtps_epi32 (out of range or NaN
 * -> 0x80000000) -> packs_epi32 -> packs_epi16 (saturate to int8). */
static inline int8_t q8_round_sat(float v) {
    const float r = rintf(v);               /* default FP env: round half to even */
    int32_t i;
    if (r >= -2147483648.0f && r < 2147483648.0f) i = (int32_t)r;
    else i = INT32_MIN;
    if (i > 127) i = 127;
    if (i < -128) i = -128;
    return (int8_t)i;
}

/* AVX2 branch, ggml.c:1192-1275: d = amax/127.f, id = amax ? 127.f/amax : 0 */
void oracle_quantize_row_q8_0_avx2(const float *x, void *vy, int k) {
    uint8_t *y = (uint8_t *)vy;
    const int nb = k / ORACLE_QK;
    for (int i = 0; i < nb; i++) {
        const float *xb = x + (size_t)i * ORACLE_QK;
        float amax = 0.0f;
        for (int j = 0; j < ORACLE_QK; j++) {
            const float a = fabsf(xb[j]);
            if (a > amax) amax = a;
        }
        const float d = amax / 127.f;
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        uint8_t *blk = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        wr16(blk, oracle_fp32_to_fp16(d));
        for (int j = 0; j < ORACLE_QK; j++) blk[2 + j] = (uint8_t)q8_round_sat(xb[j] * id);
    }
}

/* scalar reference, ggml.c:1097-1120: d = amax/127, id = d ? 1/d : 0, roundf */
void oracle_quantize_row_q8_0_ref(const float *x, void *vy, int k) {
    uint8_t *y = (uint8_t *)vy;
    const int nb = k / ORACLE_QK;
    for (int i = 0; i < nb; i++) {
        const float *xb = x + (size_t)i * ORACLE_QK;
        float amax = 0.0f;
        for (int j = 0; j < ORACLE_QK; j++) {
            const float a = fabsf(xb[j]);
            amax = amax > a ? amax : a;
        }
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        uint8_t *blk = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        wr16(blk, oracle_fp32_to_fp16(d));
        for (int j = 0; j < ORACLE_QK; j++) blk[2 + j] = (uint8_t)(int8_t)roundf(xb[j] * id);
    }
}

/* ------------------------------------------------------------------------ */
/* A6: q4_0 . q8_0 dot product. */

/* signed int8 product as the AVX2 sign trick computes it (ggml.c:660-672):
 * |w| * sign(v, w); identical to w*v except for v == -128 with w < 0. */
static inline int avx2_prod(int w, int v) {
    if (w == 0) return 0;
    int sv = (w < 0) ? (v == -128 ? -128 : -v) : v;
    return (w < 0 ? -w : w) * sv;
}

/* AVX2 order, ggml.c:2412-2435: 8 fp32 lanes; lane l accumulates
 * fma(d_x*d_y, float(sum of products of bytes 4l..4l+3), acc_l) over blocks;
 * then hsum_float_8 (ggml.c:591-597) = ((a4+a0)+(a6+a2)) + ((a5+a1)+(a7+a3)). */
float oracle_vec_dot_q4_0_q8_0_avx2(int n, const void *vx, const void *vy) {
    const uint8_t *x = (const uint8_t *)vx;
    const uint8_t *y = (const uint8_t *)vy;
    const int nb = n / ORACLE_QK;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < nb; i++) {
        const uint8_t *bx = x + (size_t)i * ORACLE_Q4_0_BLOCK_BYTES;
        const uint8_t *by = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        const float d = oracle_fp16_to_fp32(rd16(bx)) * oracle_fp16_to_fp32(rd16(by));
        for (int l = 0; l < 8; l++) {
            int s = 0;
            for (int b = 4 * l; b < 4 * l + 4; b++) {
                const int nib = b < 16 ? (bx[2 + b] & 0x0F) : (bx[2 + b - 16] >> 4);
                s += avx2_prod(nib - 8, (int8_t)by[2 + b]);
            }
            acc[l] = fmaf(d, (float)s, acc[l]);
        }
    }
    const float r0 = acc[4] + acc[0], r1 = acc[5] + acc[1];
    const float r2 = acc[6] + acc[2], r3 = acc[7] + acc[3];
    return (r0 + r2) + (r1 + r3);
}

/* scalar order, ggml.c:2588-2606: sumf += (float)sumi*dx*dy, blocks in order */
float oracle_vec_dot_q4_0_q8_0_scalar(int n, const void *vx, const void *vy) {
    const uint8_t *x = (const uint8_t *)vx;
    const uint8_t *y = (const uint8_t *)vy;
    const int nb = n / ORACLE_QK;
    float sumf = 0.0f;
    for (int i = 0; i < nb; i++) {
        const uint8_t *bx = x + (size_t)i * ORACLE_Q4_0_BLOCK_BYTES;
        const uint8_t *by = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        int sumi = 0;
        for (int j = 0; j < ORACLE_QK / 2; j++) {
            const int v0 = (bx[2 + j] & 0x0F) - 8;
            const int v1 = (bx[2 + j] >> 4) - 8;
            sumi += v0 * (int8_t)by[2 + j] + v1 * (int8_t)by[2 + j + ORACLE_QK / 2];
        }
        const float t = (float)sumi * oracle_fp16_to_fp32(rd16(bx));
        sumf += t * oracle_fp16_to_fp32(rd16(by));
    }
    return sumf;
}

/* ------------------------------------------------------------------------ */
/* AVX2 SIMD versions (CPU baseline speed).  Same arithmetic as the emulations. */

#if defined(__x86_64__)
int oracle_have_avx2(void) {
    static int cached = -1;
    if (cached < 0) {
        __builtin_cpu_init();
        cached = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") &&
                 __builtin_cpu_supports("f16c");
    }
    return cached;
}

#define AVX2_FN __attribute__((target("avx2,fma,f16c")))

AVX2_FN void oracle_quantize_row_q8_0_avx2_simd(const float *x, void *vy, int k) {
    uint8_t *y = (uint8_t *)vy;
    const int nb = k / ORACLE_QK;
    const __m256 absmask = _mm256_castsi256_ps(_mm256_set1_epi32(0x7FFFFFFF));
    const __m256i fix = _mm256_setr_epi32(0, 4, 1, 5, 2, 6, 3, 7);
    for (int i = 0; i < nb; i++) {
        const float *xb = x + (size_t)i * ORACLE_QK;
        const __m256 v0 = _mm256_loadu_ps(xb), v1 = _mm256_loadu_ps(xb + 8);
        const __m256 v2 = _mm256_loadu_ps(xb + 16), v3 = _mm256_loadu_ps(xb + 24);
        __m256 m = _mm256_max_ps(_mm256_max_ps(_mm256_and_ps(v0, absmask), _mm256_and_ps(v1, absmask)),
                                 _mm256_max_ps(_mm256_and_ps(v2, absmask), _mm256_and_ps(v3, absmask)));
        __m128 m4 = _mm_max_ps(_mm256_castps256_ps128(m), _mm256_extractf128_ps(m, 1));
        m4 = _mm_max_ps(m4, _mm_movehl_ps(m4, m4));
        m4 = _mm_max_ss(m4, _mm_shuffle_ps(m4, m4, 1));
        const float amax = _mm_cvtss_f32(m4);
        const float d = amax / 127.f;
        uint8_t *blk = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        wr16(blk, (uint16_t)_cvtss_sh(d, 0));
        const __m256 s = _mm256_set1_ps((amax != 0.0f) ? 127.f / amax : 0.0f);
        const int rm = _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC;
        const __m256i i0 = _mm256_cvtps_epi32(_mm256_round_ps(_mm256_mul_ps(v0, s), rm));
        const __m256i i1 = _mm256_cvtps_epi32(_mm256_round_ps(_mm256_mul_ps(v1, s), rm));
        const __m256i i2 = _mm256_cvtps_epi32(_mm256_round_ps(_mm256_mul_ps(v2, s), rm));
        const __m256i i3 = _mm256_cvtps_epi32(_mm256_round_ps(_mm256_mul_ps(v3, s), rm));
        const __m256i b = _mm256_packs_epi16(_mm256_packs_epi32(i0, i1), _mm256_packs_epi32(i2, i3));
        _mm256_storeu_si256((__m256i *)(blk + 2), _mm256_permutevar8x32_epi32(b, fix));
    }
}

AVX2_FN float oracle_vec_dot_q4_0_q8_0_avx2_simd(int n, const void *vx, const void *vy) {
    const uint8_t *x = (const uint8_t *)vx;
    const uint8_t *y = (const uint8_t *)vy;
    const int nb = n / ORACLE_QK;
    const __m256i lo4 = _mm256_set1_epi8(0x0F);
    const __m256i eight = _mm256_set1_epi8(8);
    const __m256i one16 = _mm256_set1_epi16(1);
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < nb; i++) {
        const uint8_t *bx = x + (size_t)i * ORACLE_Q4_0_BLOCK_BYTES;
        const uint8_t *by = y + (size_t)i * ORACLE_Q8_0_BLOCK_BYTES;
        const float d = _cvtsh_ss(rd16(bx)) * _cvtsh_ss(rd16(by));
        const __m128i q = _mm_loadu_si128((const __m128i *)(bx + 2));
        const __m256i nib = _mm256_and_si256(
            _mm256_inserti128_si256(_mm256_castsi128_si256(q), _mm_srli_epi16(q, 4), 1), lo4);
        const __m256i w = _mm256_sub_epi8(nib, eight);
        const __m256i v = _mm256_loadu_si256((const __m256i *)(by + 2));
        const __m256i p16 = _mm256_maddubs_epi16(_mm256_sign_epi8(w, w), _mm256_sign_epi8(v, w));
        const __m256 p = _mm256_cvtepi32_ps(_mm256_madd_epi16(p16, one16));
        acc = _mm256_fmadd_ps(_mm256_set1_ps(d), p, acc);
    }
    __m128 r = _mm_add_ps(_mm256_extractf128_ps(acc, 1), _mm256_castps256_ps128(acc));
    r = _mm_add_ps(r, _mm_movehl_ps(r, r));
    r = _mm_add_ss(r, _mm_movehdup_ps(r));
    return _mm_cvtss_f32(r);
}
#else
int oracle_have_avx2(void) { return 0; }
void oracle_quantize_row_q8_0_avx2_simd(const float *x, void *y, int k) { oracle_quantize_row_q8_0_avx2(x, y, k); }
float oracle_vec_dot_q4_0_q8_0_avx2_simd(int n, const void *x, const void *y) { return oracle_vec_dot_q4_0_q8_0_avx2(n, x, y); }
#endif

/* ------------------------------------------------------------------------ */
/* A10: mul_mat_q_f32 (ggml.c:11353-11411).  INIT (q8_0 of every src1 row into
 * wdata) runs on ONE thread as in ggml_graph_compute_thread (ggml.c:17113-17116);
 * COMPUTE splits the M weight rows into nth ranges of dr = ceil(M/nth). */

typedef struct {
    const uint8_t *W; const uint8_t *xq; float *y;
    int K, M, N, mode, ith, nth;
} mm_task;

static void mm_compute(const mm_task *t) {
    const size_t wrow = (size_t)(t->K / ORACLE_QK) * ORACLE_Q4_0_BLOCK_BYTES;
    const size_t xrow = (size_t)(t->K / ORACLE_QK) * ORACLE_Q8_0_BLOCK_BYTES;
    const int dr = (t->M + t->nth - 1) / t->nth;
    const int ir0 = dr * t->ith;
    const int ir1 = ir0 + dr < t->M ? ir0 + dr : t->M;
    const int simd = t->mode == 0 && oracle_have_avx2();
    for (int ir = ir0; ir < ir1; ir++) {
        const uint8_t *wr = t->W + (size_t)ir * wrow;
        for (int ic = 0; ic < t->N; ic++) {
            const uint8_t *xr = t->xq + (size_t)ic * xrow;
            float v;
            if (simd) v = oracle_vec_dot_q4_0_q8_0_avx2_simd(t->K, wr, xr);
            else if (t->mode == 0) v = oracle_vec_dot_q4_0_q8_0_avx2(t->K, wr, xr);
            else v = oracle_vec_dot_q4_0_q8_0_scalar(t->K, wr, xr);
            t->y[(size_t)ic * t->M + ir] = v;
        }
    }
}

static void *mm_thread(void *arg) { mm_compute((const mm_task *)arg); return NULL; }

/* persistent pool: workers spin on a generation counter (like ggml's
 * spin/yield loop) and run mm_compute for their slice. */
#define POOL_MAX 256
static struct {
    int nth;
    pthread_t th[POOL_MAX];
    mm_task task[POOL_MAX];
    atomic_int gen;
    atomic_int done;
    atomic_int quit;
} g_pool;

static void *pool_worker(void *arg) {
    const int ith = (int)(intptr_t)arg;
    int seen = 0;
    for (;;) {
        int g;
        while ((g = atomic_load_explicit(&g_pool.gen, memory_order_acquire)) == seen) {
            if (atomic_load_explicit(&g_pool.quit, memory_order_relaxed)) return NULL;
            sched_yield();
        }
        seen = g;
        mm_compute(&g_pool.task[ith]);
        atomic_fetch_add_explicit(&g_pool.done, 1, memory_order_release);
    }
}

void oracle_pool_shutdown(void) {
    if (g_pool.nth <= 1) { g_pool.nth = 0; return; }
    atomic_store(&g_pool.quit, 1);
    for (int i = 1; i < g_pool.nth; i++) pthread_join(g_pool.th[i], NULL);
    g_pool.nth = 0;
    atomic_store(&g_pool.quit, 0);
}

static void pool_ensure(int nth) {
    if (g_pool.nth == nth) return;
    oracle_pool_shutdown();
    atomic_store(&g_pool.gen, 0);
    g_pool.nth = nth;
    for (int i = 1; i < nth; i++) pthread_create(&g_pool.th[i], NULL, pool_worker, (void *)(intptr_t)i);
}

int oracle_mul_mat_q4_0_f32(const void *W, int K, int M, const float *x, int N,
                            float *y, int nthreads, int mode, int pool) {
    if (K % ORACLE_QK != 0 || M <= 0 || N <= 0 || nthreads < 1 || nthreads > POOL_MAX) return -1;
    const size_t xrow = (size_t)(K / ORACLE_QK) * ORACLE_Q8_0_BLOCK_BYTES;
    uint8_t *xq = (uint8_t *)malloc(xrow * (size_t)N);
    if (!xq) return -2;
    for (int n = 0; n < N; n++) {   /* INIT, single thread */
        const float *xr = x + (size_t)n * K;
        if (mode == 0 && oracle_have_avx2()) oracle_quantize_row_q8_0_avx2_simd(xr, xq + n * xrow, K);
        else if (mode == 0) oracle_quantize_row_q8_0_avx2(xr, xq + n * xrow, K);
        else oracle_quantize_row_q8_0_ref(xr, xq + n * xrow, K);
    }
    mm_task base = {(const uint8_t *)W, xq, y, K, M, N, mode, 0, nthreads};
    if (nthreads == 1) {
        mm_compute(&base);
    } else if (!pool) {
        pthread_t th[POOL_MAX];
        mm_task tk[POOL_MAX];
        for (int i = 0; i < nthreads; i++) { tk[i] = base; tk[i].ith = i; }
        for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, mm_thread, &tk[i]);
        mm_compute(&tk[0]);
        for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
    } else {
        pool_ensure(nthreads);
        for (int i = 0; i < nthreads; i++) { g_pool.task[i] = base; g_pool.task[i].ith = i; }
        atomic_store(&g_pool.done, 0);
        atomic_fetch_add_explicit(&g_pool.gen, 1, memory_order_release);
        mm_compute(&g_pool.task[0]);
        while (atomic_load_explicit(&g_pool.done, memory_order_acquire) < nthreads - 1) sched_yield();
    }
    free(xq);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* splitmix64 + Box-Muller (SURVEY.md §8d synthetic inputs) */

static inline uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_fill_gaussian(float *dst, size_t n, uint64_t seed, float mean, float std) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; i += 2) {
        /* u1 in (0,1], u2 in [0,1) from 53-bit mantissas */
        const double u1 = ((double)(splitmix64(&s) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
        const double r = sqrt(-2.0 * log(u1));
        const double a = 6.283185307179586 * u2;
        dst[i] = (float)(mean + std * r * cos(a));
        if (i + 1 < n) dst[i + 1] = (float)(mean + std * r * sin(a));
    }
}
