/*
 * q4_0_oracle.h — CPU restatement of the reference ggml q4_0 x q8_0 mul_mat path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * backend in llama.cpp-q_4_0_amd/ and the timed CPU baseline of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product (libggml_hip.so) never links or calls it.
 *
 * Every function restates one reference function (file:line under the
 * reference tree, ggml.c of Fcucgvhhhvjv/llama.cpp-q_4_0):
 *
 *   oracle_fp32_to_fp16 / oracle_fp16_to_fp32   ggml.c:284-300 (F16C, RNE), 350-397
 *   oracle_quantize_row_q4_0                    ggml.c:918-953  (A3)
 *   oracle_quantize_q4_0                        ggml.c:19157-19178 (A3 + histogram)
 *   oracle_dequantize_row_q4_0                  ggml.c:1500-1518 (A4)
 *   oracle_quantize_row_q8_0_avx2               ggml.c:1192-1275 (A5, AVX2 branch)
 *   oracle_quantize_row_q8_0_ref                ggml.c:1097-1120 (A5, scalar reference)
 *   oracle_vec_dot_q4_0_q8_0_avx2               ggml.c:2412-2435 + 591-597 (A6, AVX2 order)
 *   oracle_vec_dot_q4_0_q8_0_scalar             ggml.c:2588-2606 (A6, scalar order)
 *   oracle_mul_mat_q4_0_f32                     ggml.c:11353-11411 (A10 INIT + COMPUTE)
 *
 * Parity is pinned against the compiled reference (oracle/_ref, built from
 * /root/reference/ggml.c by oracle/Makefile) and against the golden fixtures in
 * tests/golden/ generated from it (tests/golden/gen_golden.c).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_QK 32
#define ORACLE_Q4_0_BLOCK_BYTES 18   /* sizeof(block_q4_0), ggml.c:870-875 */
#define ORACLE_Q8_0_BLOCK_BYTES 34   /* sizeof(block_q8_0), ggml.c:902-907 */

uint16_t oracle_fp32_to_fp16(float f);
float    oracle_fp16_to_fp32(uint16_t h);

void   oracle_quantize_row_q4_0(const float *x, void *y, int k);
size_t oracle_quantize_q4_0(const float *src, void *dst, int n, int k, int64_t *hist);
void   oracle_dequantize_row_q4_0(const void *x, float *y, int k);

void   oracle_quantize_row_q8_0_avx2(const float *x, void *y, int k);
void   oracle_quantize_row_q8_0_ref(const float *x, void *y, int k);

float  oracle_vec_dot_q4_0_q8_0_avx2(int n, const void *x, const void *y);
float  oracle_vec_dot_q4_0_q8_0_scalar(int n, const void *x, const void *y);

/* SIMD (AVX2/FMA/F16C) implementations of the two AVX2-branch functions, used
 * by the CPU baseline.  Bit-identical to the portable emulations above (tested).
 * Return 0 when the host CPU lacks AVX2/FMA/F16C (callers fall back). */
int    oracle_have_avx2(void);
void   oracle_quantize_row_q8_0_avx2_simd(const float *x, void *y, int k);
float  oracle_vec_dot_q4_0_q8_0_avx2_simd(int n, const void *x, const void *y);

/* A10: y[n*M + m] = vec_dot(W row m, q8_0(x row n)).
 *   mode 0: AVX2 semantics (SIMD when available, else emulation)
 *   mode 1: scalar-reference semantics (scalar q8 quantizer + scalar dot)
 * nthreads >= 1.  pool: 0 = spawn/join threads on every call like
 * ggml_graph_compute (ggml.c:17540-17571); 1 = persistent pool. */
int    oracle_mul_mat_q4_0_f32(const void *W, int K, int M, const float *x, int N,
                               float *y, int nthreads, int mode, int pool);
void   oracle_pool_shutdown(void);

/* Synthetic data: splitmix64 + Box-Muller, N(mean, std).  Deterministic. */
void   oracle_fill_gaussian(float *dst, size_t n, uint64_t seed, float mean, float std);

#ifdef __cplusplus
}
#endif
