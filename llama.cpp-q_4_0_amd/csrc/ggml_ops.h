// ggml_ops.h — launchers of the non-matmul ggml ops (ggml_ops.hip).
// All pointers are device pointers; strides are in bytes unless named ld*.  Internal to
// libggml_hip.so: the boundary is ggml_hip_compute_forward (include/ggml-hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghip {

hipError_t op_add_f32(const float *a, const float *b, float *d, int64_t n, hipStream_t s);
// d[r][c] = a[r][c] * b[row of b that row r repeats][c]; a, b, d contiguous
hipError_t op_mul_f32(const float *a, const float *b, float *d, int64_t ne00, int64_t ne01, int64_t ne02, int64_t ne03,
                      int64_t ne11, int64_t ne12, int64_t ne13, hipStream_t s);
// table: 65536 fp16 bits, ggml's table_silu_f16 / table_exp_f16 (built on the host, same formula)
hipError_t op_silu_f32(const float *x, float *d, int64_t n, const uint16_t *table, hipStream_t s);
hipError_t op_scale_f32(const float *x, float *d, float v, int64_t n, hipStream_t s);
hipError_t op_diag_mask_inf_f32(const float *x, float *d, int64_t ncols, int64_t nrows, int64_t rows_per_channel,
                                int n_past, hipStream_t s);
hipError_t op_rms_norm_f32(const float *x, float *d, int64_t ncols, int64_t nrows, int64_t ldx, int64_t ldd,
                           hipStream_t s);
hipError_t op_soft_max_f32(const float *x, float *d, int64_t ncols, int64_t nrows, const uint16_t *table, hipStream_t s);
// mode-0 rope; cs = float2 (cos, sin) [ne[2] tokens][npairs = ne[0]/2], row 0 = position n_past
hipError_t op_rope_f32(const void *x, void *d, const int64_t ne[4], const int64_t nbx[4], const int64_t nbd[4],
                       const void *cs, int npairs, hipStream_t s);
hipError_t op_cpy_f32(const void *x, void *d, bool to_f16, int64_t n, int64_t ne00, int64_t ne01, int64_t nb00,
                      int64_t nb01, int64_t nb02, int64_t ne10, int64_t ne11, int64_t nb10, int64_t nb11, int64_t nb12,
                      hipStream_t s);
// dst [ne02][ne11][ne01] f32 contiguous = src0 f16 rows (K, strides nb01/nb02) . fp16(src1 f32 rows)
// merged != nullptr: also the contiguous copy of permute(dst, 0, 2, 1, 3) (fused KQV_merged_contiguous)
hipError_t op_mul_mat_f16_f32(const void *s0, const void *s1, float *d, int K, int64_t ne01, int64_t ne11, int64_t ne02,
                              int64_t nb01, int64_t nb02, int64_t nb11, int64_t nb12, hipStream_t s,
                              float *merged = nullptr, int tiled = -1);   // tiled: -1 auto (bitwise kernels), 0 / 1 force those;
                              // 2 the fast-mode MFMA kernel, -2 auto with it (ne11 >= 32)
// rope (as op_rope_f32) whose output is then copied (ggml_cpy, F32 -> F32/F16) into the strided view c
hipError_t op_rope_cpy_f32(const void *x, void *d, const int64_t ne[4], const int64_t nbx[4], const int64_t nbd[4],
                           const void *cs, int npairs, void *c, bool to_f16, int64_t ne10, int64_t ne11, int64_t nb10,
                           int64_t nb11, int64_t nb12, hipStream_t s);

// independent rope / rope->cpy / cpy nodes in one launch (each element as its own op computes it)
constexpr int ELEM_MAX = 4;
struct ElemOp {
    int kind;              // 0 rope (mode 0; then the copy into c when c != nullptr), 1 cpy x -> c
                           // (set by op_elem_batch: 2 the transposed 2-d cpy in 64 x 64 LDS tiles,
                           // 3 a rope on two pairs per thread)
    int f16;               // the copy's target is F16 (else F32)
    int pack;              // set by op_elem_batch (kind 3): a thread's 4 copied values share a target row
    const char *x;         // source
    char *d;               // rope output
    char *c;               // copy target (strided view) or nullptr
    const float2 *cs;      // rope (cos, sin) rows from position n_past
    int npairs;
    int64_t n;             // work items: rope pairs or copied elements
    int64_t ne0, ne1, ne2;                 // rope: x/d shape; cpy: ne00, ne01 (ne2 unused)
    int64_t nbx1, nbx2, nbx3;              // rope: x strides 1..3; cpy: nb00, nb01, nb02
    int64_t nbd1, nbd2, nbd3;              // rope: d strides 1..3
    int64_t ne10, ne11, nb10, nb11, nb12;  // the copy target's shape / strides
};
struct ElemBatch {
    ElemOp op[ELEM_MAX];
    int nops;
    unsigned block_begin[ELEM_MAX];       // filled by op_elem_batch
};
hipError_t op_elem_batch(const ElemBatch &b, hipStream_t s);

// fused chains (each stage bit-identical to its own op above; intermediates stored unless nullptr)
// [sum = a + b] -> norm = rms_norm(sum) -> out = norm * w (w: one row); a == nullptr: rms_norm(b)
hipError_t op_add_rms_norm_mul_f32(const float *a, const float *b, float *sum, float *norm, const float *w, float *out,
                                   int64_t ncols, int64_t nrows, hipStream_t s);
// scaled = x * v -> masked = diag_mask_inf(scaled, n_past) -> d = soft_max(masked)
hipError_t op_scale_mask_soft_max_f32(const float *x, float *scaled, float *masked, float *d, float v, int64_t ncols,
                                      int64_t nrows, int64_t rows_per_channel, int n_past, const uint16_t *table,
                                      hipStream_t s);
// decode attention's second half, one query row per head: scaled/masked/sm = scale -> diag_mask_inf
// -> soft_max of kq's rows (as op_scale_mask_soft_max_f32), kqv (+ merged) = V.fp16(sm) (as
// op_mul_mat_f16_f32 with N = 1); V^T rows of nkv f16 at nb01v, heads at nb02v; nullptr = not stored
hipError_t op_softmax_kqv(const float *kq, float *scaled, float *masked, float *sm, float v, int n_past,
                          const uint16_t *table, int64_t nkv, int64_t nhead, const void *vs, int64_t nb01v, int64_t nb02v,
                          int64_t nout, float *kqv, float *merged, hipStream_t s);
// the whole decode attention of one query row per head: KQ = K.fp16(q) per head (as op_mul_mat_f16_f32 with
// N = 1: K rows f16 at nb01k, heads at nb02k; q heads at nb02q, hd <= 256) into LDS, then as op_softmax_kqv;
// kq / scaled / masked / sm stored by each head's first workgroup unless nullptr (pass one pointer per
// buffer: the last tensor of an in-place chain)
hipError_t op_kq_softmax_kqv(const void *ks, int64_t nb01k, int64_t nb02k, const float *q, int64_t nb02q, int hd,
                             float *kq, float *scaled, float *masked, float *sm, float v, int n_past, const uint16_t *table,
                             int64_t nkv, int64_t nhead, const void *vs, int64_t nb01v, int64_t nb02v, int64_t nout,
                             float *kqv, float *merged, hipStream_t s);
// u = silu(a) -> out = u * b (same shape)
// mismatches of the direct silu / exp evaluation against the host tables over every finite fp16 input
// (bad_dev: two zeroed ints on the device; q4_0_device.h lut_silu / lut_exp)
hipError_t op_lut_check(const uint16_t *silu, const uint16_t *ex, int *bad_dev, hipStream_t s);
hipError_t op_silu_mul_f32(const float *a, const float *b, float *u, float *out, int64_t n, const uint16_t *table,
                           hipStream_t s);
// The same chains with the k_gemm9 x image of out written beside it into xws (codes [nb][3][Np][16 B] +
// fp16 d_x [nb][Np], nb = ncols / 32; bitwise what gemm9_prep_x makes of out).  ncols % 64 == 0,
// ncols <= 16384, 16-byte aligned operands; hipErrorInvalidValue otherwise (nothing launched).
bool op_x9_ok(int64_t ncols, int64_t nrows);
hipError_t op_add_rms_norm_mul_f32_x9(const float *a, const float *b, float *sum, float *norm, const float *w, float *out,
                                      int64_t ncols, int64_t nrows, void *xws, int64_t Np, hipStream_t s);
hipError_t op_silu_mul_f32_x9(const float *a, const float *b, float *u, float *out, int64_t ncols, int64_t nrows,
                              const uint16_t *table, void *xws, int64_t Np, hipStream_t s);

}  // namespace ghip
