// ggml_ops.hip — gfx950 kernels for the non-matmul ggml ops of a fully offloaded LLaMA layer
// (SURVEY.md §8f row 4), each a restatement of the reference's CPU op so that a graph run on the
// device reproduces ggml.c's results bit for bit:
//
//   add_f32          ggml_compute_forward_add_f32      ggml.c:8260   dst = a + b
//   mul_f32          ggml_compute_forward_mul_f32      ggml.c:9149   dst = a * b (b rows broadcast)
//   silu_f32         ggml_vec_silu_f32 (GGML_SILU_FP16) ggml.c:3531  y = table_silu_f16[fp16(x)]
//   rms_norm_f32     ggml_compute_forward_rms_norm_f32 ggml.c:10389  double sum of x*x, eps 1e-6
//   rope_f32         ggml_compute_forward_rope_f32     ggml.c:12714  mode 0; cos/sin from a host table
//   diag_mask_inf    ggml_compute_forward_diag_mask_f32 ggml.c:12195
//   soft_max_f32     ggml_compute_forward_soft_max_f32 ggml.c:12284  fp16 exp table, double sum
//   scale_f32        ggml_compute_forward_scale_f32    ggml.c:11633
//   cpy_f32_{f32,f16} ggml_compute_forward_dup (strided), GGML_FP32_TO_FP16 = RNE
//   mul_mat_f16_f32  ggml_compute_forward_mul_mat_f16_f32 ggml.c:11026 + ggml_vec_dot_f16 ggml.c:2303
//                    (src1 rounded to fp16, the AVX F16 lane schedule and reduction order)
//
// The transcendental parts (silu, exp, cos/sin) are NOT evaluated on the device: ggml.c itself
// evaluates silu and exp through 64 K-entry fp16 tables built with the host libm (ggml.c:4246-4254),
// and rope's cos/sin are host libm values too; the backend builds the same tables on the host
// (ggml-hip-ops.cpp) and the kernels look them up.  All other arithmetic is IEEE single/double in the
// CPU's order (built with -ffp-contract=off; the sums the CPU forms in double are formed in double).
// These are small, latency-bound launches (a decode layer moves a few KB through them); one wave
// per row where the CPU reduces over a row, one lane per element otherwise.
#include "ggml_ops.h"
#include "launch.h"
#include "q4_0_device.h"

#include <cmath>

namespace ghip {

namespace {

__device__ __forceinline__ float h2f_bits(uint16_t b) {
    _Float16 h;
    __builtin_memcpy(&h, &b, 2);
    return (float)h;
}
__device__ __forceinline__ uint16_t f2h_bits(float f) {
    asm volatile("" : "+v"(f));           // keep hipcc from folding into v_fma_mix (sign of zero)
    const _Float16 h = (_Float16)f;       // v_cvt_f16_f32: round to nearest even (F16C _cvtss_sh(x, 0))
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

constexpr int TPB = 256;

inline unsigned blocks(int64_t n, int per = TPB) { return (unsigned)((n + per - 1) / per); }

// ----------------------------------------------------------------------------------- elementwise
__global__ __launch_bounds__(TPB) void k_add_f32(const float *a, const float *b, float *d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < n) d[i] = a[i] + b[i];
}

// src0/dst contiguous [ne03][ne02][ne01][ne00]; src1 contiguous [ne13][ne12][ne11][ne00], repeated
__global__ __launch_bounds__(TPB) void k_mul_f32(const float *a, const float *b, float *d, int64_t ne00, int64_t ne01,
                                                 int64_t ne02, int64_t nrows, int64_t ne11, int64_t ne12, int64_t ne13) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= nrows * ne00) return;
    const int64_t r = i / ne00, c = i - r * ne00;
    const int64_t i03 = r / (ne02 * ne01), i02 = (r / ne01) % ne02, i01 = r % ne01;
    const int64_t rb = ((i03 % ne13) * ne12 + (i02 % ne12)) * ne11 + (i01 % ne11);
    d[i] = a[i] * b[rb * ne00 + c];
}

__global__ __launch_bounds__(TPB) void k_silu_f32(const float *x, float *d, int64_t n, const uint16_t *table) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < n) d[i] = h2f_bits(lut_silu(table, f2h_bits(x[i])));
}

__global__ __launch_bounds__(TPB) void k_scale_f32(const float *x, float *d, float v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < n) d[i] = x[i] * v;
}

// rows [nrows][ncols] with row r in channel r / rows_per_channel at row j = r % rows_per_channel:
// element i of row j becomes -inf when i > n_past + j (and i >= n_past, which that implies)
__global__ __launch_bounds__(TPB) void k_diag_mask_inf_f32(const float *x, float *d, int64_t ncols, int64_t n,
                                                           int64_t rows_per_channel, int n_past) {
    const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= n) return;
    const int64_t r = k / ncols, i = k - r * ncols, j = r % rows_per_channel;
    d[k] = i > n_past + j ? -INFINITY : x[k];
}

// ----------------------------------------------------------------------------------- row reductions
// one wave per row: sum = (double)(x*x) over the row, mean = (float)(sum / n), scale = 1/sqrt(mean + eps)
__global__ __launch_bounds__(TPB) void k_rms_norm_f32(const float *x, float *d, int64_t ncols, int64_t nrows,
                                                      int64_t ldx, int64_t ldd) {
    const int64_t r = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const float *xr = x + r * ldx;
    double s = 0.0;
    for (int64_t i = lane; i < ncols; i += 64) {
        const float v = xr[i];
        s += (double)(v * v);
    }
    s = wave_sum_d(s);
    const float mean = (float)(s / (double)ncols);
    // (float)sqrt((double)v) is the correctly rounded sqrtf(v) (double has >= 2*24+2 bits)
    const float scale = 1.0f / (float)__builtin_sqrt((double)(mean + 1e-6f));
    float *dr = d + r * ldd;
    for (int64_t i = lane; i < ncols; i += 64) dr[i] = xr[i] * scale;
}

// one wave per row: max, then val = exp_table[fp16(x - max)] (0 for -inf), double sum, y = val * (float)(1/sum)
__global__ __launch_bounds__(TPB) void k_soft_max_f32(const float *x, float *d, int64_t ncols, int64_t nrows,
                                                      const uint16_t *table) {
    const int64_t r = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const float *xr = x + r * ncols;
    float *dr = d + r * ncols;
    float mx = -INFINITY;
    for (int64_t i = lane; i < ncols; i += 64) mx = fmaxf(mx, xr[i]);
    mx = wave_max_f(mx);
    double s = 0.0;
    for (int64_t i = lane; i < ncols; i += 64) {
        const float v = xr[i];
        float e = 0.0f;
        if (v != -INFINITY) {
            e = h2f_bits(lut_exp(table, f2h_bits(v - mx)));
            s += (double)e;
        }
        dr[i] = e;
    }
    s = wave_sum_d(s);
    const float inv = (float)(1.0 / s);
    for (int64_t i = lane; i < ncols; i += 64) dr[i] = dr[i] * inv;
}

// ----------------------------------------------------------------------------------- rope (mode 0)
// x/d: [ne3][ne2][ne1][ne0] with byte strides; token i2 uses position p = n_past + i2, pair j of a row
// uses cs[(p - p0) * npairs + j] = (cos, sin) of theta_j (host libm, theta_j = p * theta_scale^j by
// repeated float multiplication as ggml.c:12814 does)
__global__ __launch_bounds__(TPB) void k_rope_f32(const char *x, char *d, int64_t ne0, int64_t ne1, int64_t ne2,
                                                  int64_t nb01, int64_t nb02, int64_t nb03, int64_t nb1, int64_t nb2,
                                                  int64_t nb3, int64_t n, const float2 *cs, int npairs) {
    const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= n) return;
    const int64_t np = ne0 / 2;
    const int64_t j = k % np;
    const int64_t r = k / np;
    const int64_t i1 = r % ne1, i2 = (r / ne1) % ne2, i3 = r / (ne1 * ne2);
    const float2 t = cs[i2 * npairs + j];
    const float *s = (const float *)(x + i3 * nb03 + i2 * nb02 + i1 * nb01) + 2 * j;
    float *o = (float *)(d + i3 * nb3 + i2 * nb2 + i1 * nb1) + 2 * j;
    const float x0 = s[0], x1 = s[1];
    o[0] = x0 * t.x - x1 * t.y;
    o[1] = x0 * t.y + x1 * t.x;
}

// rope, then ggml_cpy of the rope output (contiguous [ne2][ne1][ne0]) into a strided view (the K
// cache, F16): element i = i0 + ne0*(i1 + ne1*i2) of the rope output goes to the copy's
// (i10, i11, i12) = i split by (ne10, ne11), as k_cpy_f32 maps it
template <bool F16>
__global__ __launch_bounds__(TPB) void k_rope_cpy(const char *x, char *d, int64_t ne0, int64_t ne1, int64_t ne2,
                                                  int64_t nb01, int64_t nb02, int64_t nb03, int64_t nb1, int64_t nb2,
                                                  int64_t nb3, int64_t n, const float2 *cs, int npairs, char *c,
                                                  int64_t ne10, int64_t ne11, int64_t nb10, int64_t nb11, int64_t nb12) {
    const int64_t k = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= n) return;
    const int64_t np = ne0 / 2;
    const int64_t j = k % np;
    const int64_t r = k / np;
    const int64_t i1 = r % ne1, i2 = (r / ne1) % ne2, i3 = r / (ne1 * ne2);
    const float2 t = cs[i2 * npairs + j];
    const float *src = (const float *)(x + i3 * nb03 + i2 * nb02 + i1 * nb01) + 2 * j;
    float *o = (float *)(d + i3 * nb3 + i2 * nb2 + i1 * nb1) + 2 * j;
    const float x0 = src[0], x1 = src[1];
    const float y0 = x0 * t.x - x1 * t.y;
    const float y1 = x0 * t.y + x1 * t.x;
    o[0] = y0;
    o[1] = y1;
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int64_t i = 2 * j + e + ne0 * (i1 + ne1 * i2);
        const int64_t i12 = i / (ne10 * ne11), i11 = (i / ne10) % ne11, i10 = i % ne10;
        char *dst = c + i10 * nb10 + i11 * nb11 + i12 * nb12;
        const float v = e ? y1 : y0;
        if (F16)
            *(uint16_t *)dst = f2h_bits(v);
        else
            *(float *)dst = v;
    }
}

// ----------------------------------------------------------------------------------- cpy (strided)
template <bool F16>
__global__ __launch_bounds__(TPB) void k_cpy_f32(const char *x, char *d, int64_t n, int64_t ne00, int64_t ne01,
                                                 int64_t nb00, int64_t nb01, int64_t nb02, int64_t ne10, int64_t ne11,
                                                 int64_t nb10, int64_t nb11, int64_t nb12) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const int64_t i02 = i / (ne00 * ne01), i01 = (i / ne00) % ne01, i00 = i % ne00;
    const int64_t i12 = i / (ne10 * ne11), i11 = (i / ne10) % ne11, i10 = i % ne10;
    const float v = *(const float *)(x + i00 * nb00 + i01 * nb01 + i02 * nb02);
    char *o = d + i10 * nb10 + i11 * nb11 + i12 * nb12;
    if (F16)
        *(uint16_t *)o = f2h_bits(v);
    else
        *(float *)o = v;
}

// ----------------------------------------------------------------------------------- batched
// Up to ELEM_MAX independent rope / rope->cpy / cpy nodes in one launch (the nodes a LLaMA layer
// runs between its q4_0 sibling group and the attention: rope K -> K cache, V -> V cache, rope Q).
// Each block belongs to one op (block_begin prefix sums); every element is computed by the same
// expression as the op's own kernel above.
// I: the index type of the per-element divisions (uint32_t when every op's extents fit: the 64-bit
// divisions would bound the prefill launch on the VALU; addresses stay 64-bit either way)
template <typename I>
__global__ __launch_bounds__(TPB) void k_elem_batch(const ElemBatch b) {
    int o = 0;
#pragma unroll
    for (int q = 1; q < ELEM_MAX; q++) o += (q < b.nops && blockIdx.x >= b.block_begin[q]) ? 1 : 0;
    // constant-index copies: no dynamic indexing into the kernarg struct
    ElemOp op = b.op[0];
#pragma unroll
    for (int q = 1; q < ELEM_MAX; q++)
        if (o == q) op = b.op[q];
    if (op.kind == 2) {
        // the 2-d cpy whose source runs along dim 1 and target along dim 0 (Vcur -> the transposed V
        // cache at prefill): one 64 x 64 tile per workgroup through LDS, read along the source's rows
        // and written along the target's, each value converted as kind 1 converts it
        __shared__ float tile[64][65];
        const int64_t t = blockIdx.x - b.block_begin[o];
        const int64_t nt0 = (op.ne0 + 63) / 64;
        const int64_t t0 = (t % nt0) * 64, t1 = (t / nt0) * 64;
        const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
        for (int r = ly; r < 64; r += TPB / 64) {
            const int64_t i00 = t0 + r, i01 = t1 + lx;
            if (i00 < op.ne0 && i01 < op.ne1) tile[r][lx] = *(const float *)(op.x + i00 * op.nbx1 + i01 * 4);
        }
        __syncthreads();
        for (int r = ly; r < 64; r += TPB / 64) {
            const int64_t i00 = t0 + lx, i01 = t1 + r;
            if (i00 < op.ne0 && i01 < op.ne1) {
                char *dst = op.c + i00 * op.nb10 + i01 * op.nb11;
                if (op.f16)
                    *(uint16_t *)dst = f2h_bits(tile[lx][r]);
                else
                    *(float *)dst = tile[lx][r];
            }
        }
        return;
    }
    const int64_t k = (int64_t)(blockIdx.x - b.block_begin[o]) * TPB + threadIdx.x;
    if (k >= op.n) return;
    if (op.kind == 1) {                                   // cpy, as k_cpy_f32
        const I i = (I)k, ne0 = (I)op.ne0, ne1 = (I)op.ne1, ne10 = (I)op.ne10, ne11 = (I)op.ne11;
        const int64_t i02 = i / (ne0 * ne1), i01 = (i / ne0) % ne1, i00 = i % ne0;
        const int64_t i12 = i / (ne10 * ne11), i11 = (i / ne10) % ne11, i10 = i % ne10;
        const float v = *(const float *)(op.x + i00 * op.nbx1 + i01 * op.nbx2 + i02 * op.nbx3);
        char *dst = op.c + i10 * op.nb10 + i11 * op.nb11 + i12 * op.nb12;
        if (op.f16)
            *(uint16_t *)dst = f2h_bits(v);
        else
            *(float *)dst = v;
        return;
    }
    if (op.kind == 3) {
        // kind 0 on two pairs per thread (set by op_elem_batch when every row and the (cos, sin) rows
        // are 16-byte aligned): the same products per pair, 16-byte loads and stores, and the four
        // values' copy in one 8- (F16) or 16-byte (F32) store when they share a contiguous row (pack)
        const I nq = (I)(op.ne0 / 4), ne1 = (I)op.ne1, ne2 = (I)op.ne2;
        const I q = (I)k % nq, r = (I)k / nq;
        const int64_t i1 = r % ne1, i2 = (r / ne1) % ne2, i3 = r / (ne1 * ne2);
        const float4 t = *(const float4 *)(op.cs + i2 * op.npairs + 2 * q);
        const float4 x = *(const float4 *)(op.x + i3 * op.nbx3 + i2 * op.nbx2 + i1 * op.nbx1 + 16 * (int64_t)q);
        float4 y;
        y.x = x.x * t.x - x.y * t.y;
        y.y = x.x * t.y + x.y * t.x;
        y.z = x.z * t.z - x.w * t.w;
        y.w = x.z * t.w + x.w * t.z;
        *(float4 *)(op.d + i3 * op.nbd3 + i2 * op.nbd2 + i1 * op.nbd1 + 16 * (int64_t)q) = y;
        if (op.c) {
            const I ne10 = (I)op.ne10, ne11 = (I)op.ne11;
            const I i = 4 * q + (I)op.ne0 * ((I)i1 + ne1 * (I)i2);
            const float v[4] = {y.x, y.y, y.z, y.w};
            if (op.pack) {
                const int64_t i12 = i / (ne10 * ne11), i11 = (i / ne10) % ne11, i10 = i % ne10;
                char *dst = op.c + i10 * op.nb10 + i11 * op.nb11 + i12 * op.nb12;
                if (op.f16) {
                    const uint2 h = make_uint2((uint32_t)f2h_bits(v[0]) | ((uint32_t)f2h_bits(v[1]) << 16),
                                               (uint32_t)f2h_bits(v[2]) | ((uint32_t)f2h_bits(v[3]) << 16));
                    *(uint2 *)dst = h;
                } else {
                    *(float4 *)dst = y;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const I ie = i + e;
                    const int64_t i12 = ie / (ne10 * ne11), i11 = (ie / ne10) % ne11, i10 = ie % ne10;
                    char *dst = op.c + i10 * op.nb10 + i11 * op.nb11 + i12 * op.nb12;
                    if (op.f16)
                        *(uint16_t *)dst = f2h_bits(v[e]);
                    else
                        *(float *)dst = v[e];
                }
            }
        }
        return;
    }
    // rope (mode 0), as k_rope_f32; then (c != nullptr) the copy of k_rope_cpy
    const I np = (I)(op.ne0 / 2), ne1 = (I)op.ne1, ne2 = (I)op.ne2;
    const I j = (I)k % np;
    const I r = (I)k / np;
    const int64_t i1 = r % ne1, i2 = (r / ne1) % ne2, i3 = r / (ne1 * ne2);
    const float2 t = op.cs[i2 * op.npairs + j];
    const float *src = (const float *)(op.x + i3 * op.nbx3 + i2 * op.nbx2 + i1 * op.nbx1) + 2 * j;
    float *out = (float *)(op.d + i3 * op.nbd3 + i2 * op.nbd2 + i1 * op.nbd1) + 2 * j;
    const float x0 = src[0], x1 = src[1];
    const float y0 = x0 * t.x - x1 * t.y;
    const float y1 = x0 * t.y + x1 * t.x;
    out[0] = y0;
    out[1] = y1;
    if (op.c) {
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const I ne10 = (I)op.ne10, ne11 = (I)op.ne11;
            const I i = 2 * j + e + (I)op.ne0 * ((I)i1 + ne1 * (I)i2);
            const int64_t i12 = i / (ne10 * ne11), i11 = (i / ne10) % ne11, i10 = i % ne10;
            char *dst = op.c + i10 * op.nb10 + i11 * op.nb11 + i12 * op.nb12;
            const float v = e ? y1 : y0;
            if (op.f16)
                *(uint16_t *)dst = f2h_bits(v);
            else
                *(float *)dst = v;
        }
    }
}

// ----------------------------------------------------------------------------------- f16 x f32 mul_mat
// dst[i2][i1][i0] = ggml_vec_dot_f16(K, src0[i2][i0][:], fp16(src1[i2][i1][:])), src0 rows f16
// (nb00 = 2), src1 rows f32 (nb10 = 4), arbitrary row/channel strides (the permuted K and the
// transposed V views of the KV cache).  32 lanes per output = the 4 x 8 fp32 accumulator lanes of
// the AVX F16 loop (element e < np goes to lane e % 32, fma in order of e); then GGML_F32x8_REDUCE
// (accumulators (0+2)+(1+3), 128-bit halves, two hadds) and the tail e >= np added in double.
// merged != nullptr: the value is also stored at merged[(i1 * ne02 + i2) * ne01 + i0], i.e. the
// contiguous copy of permute(dst, 0, 2, 1, 3) (llama.cpp's KQV_merged_contiguous, fused)
__global__ __launch_bounds__(TPB) void k_mul_mat_f16_f32(const char *s0, const char *s1, float *d, int K,
                                                         int64_t ne01, int64_t ne11, int64_t ne02, int64_t nb01,
                                                         int64_t nb02, int64_t nb11, int64_t nb12, float *merged) {
    const int64_t o = ((int64_t)blockIdx.x * TPB + threadIdx.x) >> 5;   // output index
    const int l = threadIdx.x & 31;
    const int64_t nout = ne01 * ne11 * ne02;
    const bool valid = o < nout;
    const int64_t oc = valid ? o : 0;
    const int64_t i0 = oc % ne01, i1 = (oc / ne01) % ne11, i2 = oc / (ne01 * ne11);
    const uint16_t *xr = (const uint16_t *)(s0 + i2 * nb02 + i0 * nb01);
    const float *yr = (const float *)(s1 + i2 * nb12 + i1 * nb11);
    const int np = K & ~31, tl = K - np, kl = K > 0 ? K - 1 : 0;
    float acc = 0.0f;
    // batches of 4 unconditional loads of clamped addresses (issued back to back; a load under a
    // branch would wait at the join), used in order of e
    for (int e0 = 0; e0 < np; e0 += 128) {
        uint16_t xb[4];
        float yb[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int e = min(e0 + l + 32 * j, kl);
            xb[j] = xr[e];
            yb[j] = yr[e];
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (e0 + l + 32 * j < np) acc = fmaf(h2f_bits(xb[j]), h2f_bits(f2h_bits(yb[j])), acc);
    }
    // the tail e >= np: each lane's product (loaded with the batches' clamping), summed below in order
    const uint16_t xt = xr[min(np + l, kl)];
    const float yt = yr[min(np + l, kl)];
    const float pt = l < tl ? h2f_bits(xt) * h2f_bits(f2h_bits(yt)) : 0.0f;
    // lane = 8*j + m: a_m = s0 + s2, b_m = s1 + s3, c_m = a_m + b_m
    const float p16 = __shfl_xor(acc, 16, 32);
    const float a = acc + p16;                                        // lanes 0-7: s0+s2, 8-15: s1+s3
    const float p8 = __shfl_xor(a, 8, 32);
    const float c = a + p8;                                           // lanes 0-7: (s0+s2)+(s1+s3)
    const float c4 = __shfl_xor(c, 4, 32);
    const float t0 = c + c4;                                          // lanes 0-3: c_k + c_{k+4}
    const float t01 = t0 + __shfl_xor(t0, 1, 32);                     // lane 0: t0_0 + t0_1, lane 2: t0_2 + t0_3
    const float t23 = __shfl(t01, 2, 32);
    const float res = t01 + t23;                                      // lane 0
    double sum = (double)res;                                         // + the tail in double, in order of e
    for (int e = 0; e < tl; e++) sum += (double)__shfl(pt, e, 32);
    if (l == 0 && valid) {
        d[o] = (float)sum;
        if (merged) merged[(i1 * ne02 + i2) * ne01 + i0] = (float)sum;
    }
}

// The same dot products for many src1 rows (prefill attention: KQ and KQV over N tokens), tiled.
// A workgroup owns FT x FT outputs of one channel i2; the four threads of a group own the four
// 8-lane AVX accumulators j = 0..3 (chains 8j..8j+7: element e < np goes to chain e % 32, fma in
// order of e) of a 4 x 4 output block, reading 8 fp16 values per row per 32-element step from LDS
// (src0 rows as stored, src1 rows rounded to fp16 on staging) and multiplying them with
// v_fma_mix_f32 (fp16 operands, exact widening, one fp32 rounding: the same value as fmaf on the
// widened operands).  Afterwards (s0+s2)+(s1+s3) comes from two quad DPP exchanges within the
// group, thread j finishes column j of the block with the in-vector tree of GGML_F32x8_REDUCE and
// the double tail: the same operations in the same order as k_mul_mat_f16_f32, so both kernels
// give the same bits.
constexpr int FT = 32;                 // outputs per tile side
constexpr int FB = 4;                  // outputs per block side (per group of 4 threads)
constexpr int FKC = 128;               // K elements per LDS stage (4 AVX steps)
constexpr int FLD = FKC + 8;           // LDS row pitch in halves (16-byte rows, staggered banks)
static_assert((FT / FB) * (FT / FB) * 4 == TPB, "one group of four threads per output block");

__device__ __forceinline__ void fma_mix_lo(uint32_t a, uint32_t b, float &c) {   // c = fp16 a.lo * b.lo + c
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void fma_mix_hi(uint32_t a, uint32_t b, float &c) {   // c = fp16 a.hi * b.hi + c
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "+v"(c) : "v"(a), "v"(b));
}
template <int CTRL>
__device__ __forceinline__ float quad_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__global__ __launch_bounds__(TPB, 2) void k_mul_mat_f16_f32_tiled(const char *s0, const char *s1, float *d, int K,
                                                               int64_t ne01, int64_t ne11, int64_t ne02, int64_t nb01,
                                                               int64_t nb02, int64_t nb11, int64_t nb12,
                                                               float *merged) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[FT * FLD];
    __shared__ __attribute__((aligned(16))) uint16_t ys[FT * FLD];
    const int t = threadIdx.x;
    const int j = t & 3, g = t >> 2;                       // accumulator group, output block
    const int br = (g & 7) * FB, bc = (g >> 3) * FB;       // block origin in the tile (rows, cols)
    const int64_t r0 = (int64_t)blockIdx.x * FT, c0 = (int64_t)blockIdx.y * FT, i2 = blockIdx.z;
    const char *x0 = s0 + i2 * nb02;
    const char *y0 = s1 + i2 * nb12;
    const int np = K & ~31;
    // staging role: rows sr and sr + 16 of the tile, 8 consecutive elements from se
    const int sr = t >> 4, se = (t & 15) * 8;
    const uint16_t *xg[2];
    const float *yg[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int64_t xr = r0 + sr + 16 * q < ne01 ? r0 + sr + 16 * q : ne01 - 1;   // clamped: loaded, not stored
        const int64_t yr = c0 + sr + 16 * q < ne11 ? c0 + sr + 16 * q : ne11 - 1;
        xg[q] = (const uint16_t *)(x0 + xr * nb01);
        yg[q] = (const float *)(y0 + yr * nb11);
    }

    float acc[FB][FB][8];
#pragma unroll
    for (int r = 0; r < FB; r++)
#pragma unroll
        for (int c = 0; c < FB; c++)
#pragma unroll
            for (int e = 0; e < 8; e++) acc[r][c][e] = 0.0f;

    // stages cover [0, K): the tail e >= np lies in the last one and is read back from LDS below
    for (int k0 = 0; k0 < K; k0 += FKC) {
        const int k = k0 + se;
        uint4 xv[2], yv[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            uint32_t xw[4], yw[4];
            if (k + 8 <= K && ((uintptr_t)(xg[q] + k) & 15) == 0) {
                const uint4 v = *reinterpret_cast<const uint4 *>(xg[q] + k);
                xw[0] = v.x, xw[1] = v.y, xw[2] = v.z, xw[3] = v.w;
            } else {
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    const uint32_t lo = k + 2 * w < K ? xg[q][k + 2 * w] : 0u;
                    const uint32_t hi = k + 2 * w + 1 < K ? xg[q][k + 2 * w + 1] : 0u;
                    xw[w] = lo | (hi << 16);
                }
            }
            float yf[8];
            if (k + 8 <= K && ((uintptr_t)(yg[q] + k) & 15) == 0) {
                const float4 a = *reinterpret_cast<const float4 *>(yg[q] + k);
                const float4 b = *reinterpret_cast<const float4 *>(yg[q] + k + 4);
                yf[0] = a.x, yf[1] = a.y, yf[2] = a.z, yf[3] = a.w, yf[4] = b.x, yf[5] = b.y, yf[6] = b.z, yf[7] = b.w;
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) yf[e] = k + e < K ? yg[q][k + e] : 0.0f;
            }
#pragma unroll
            for (int w = 0; w < 4; w++) yw[w] = (uint32_t)f2h_bits(yf[2 * w]) | ((uint32_t)f2h_bits(yf[2 * w + 1]) << 16);
            xv[q] = make_uint4(xw[0], xw[1], xw[2], xw[3]);
            yv[q] = make_uint4(yw[0], yw[1], yw[2], yw[3]);
        }
        __syncthreads();                                   // previous stage consumed
#pragma unroll
        for (int q = 0; q < 2; q++) {
            *reinterpret_cast<uint4 *>(xs + (sr + 16 * q) * FLD + se) = xv[q];
            *reinterpret_cast<uint4 *>(ys + (sr + 16 * q) * FLD + se) = yv[q];
        }
        __syncthreads();
        const int rem = np - k0;
        const int steps = rem <= 0 ? 0 : (rem / 32 < FKC / 32 ? rem / 32 : FKC / 32);
        for (int s = 0; s < steps; s++) {
            const int off = 32 * s + 8 * j;
            uint4 xr[FB];
#pragma unroll
            for (int r = 0; r < FB; r++) xr[r] = *reinterpret_cast<const uint4 *>(xs + (br + r) * FLD + off);
#pragma unroll
            for (int c = 0; c < FB; c++) {
                const uint4 yc = *reinterpret_cast<const uint4 *>(ys + (bc + c) * FLD + off);
                const uint32_t yw[4] = {yc.x, yc.y, yc.z, yc.w};
#pragma unroll
                for (int r = 0; r < FB; r++) {
                    const uint32_t xw[4] = {xr[r].x, xr[r].y, xr[r].z, xr[r].w};
#pragma unroll
                    for (int w = 0; w < 4; w++) {
                        fma_mix_lo(xw[w], yw[w], acc[r][c][2 * w]);
                        fma_mix_hi(xw[w], yw[w], acc[r][c][2 * w + 1]);
                    }
                }
            }
        }
    }
    // (s0+s2)+(s1+s3) per lane e: quad_perm [2,3,0,1] (xor 2), then [1,0,3,2] (xor 1)
#pragma unroll
    for (int r = 0; r < FB; r++)
#pragma unroll
        for (int c = 0; c < FB; c++)
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const float a = acc[r][c][e] + quad_dpp<0x4E>(acc[r][c][e]);
                acc[r][c][e] = a + quad_dpp<0xB1>(a);
            }
    // thread j finishes column j of the block
#pragma unroll
    for (int c = 0; c < FB; c++) {
        if (c != j) continue;
#pragma unroll
        for (int r = 0; r < FB; r++) {
            const float *v = acc[r][c];
            const float t0 = v[0] + v[4], t1 = v[1] + v[5], t2 = v[2] + v[6], t3 = v[3] + v[7];
            const float res = (t0 + t1) + (t2 + t3);
            const int64_t i0 = r0 + br + r, i1 = c0 + bc + c;
            if (i0 < ne01 && i1 < ne11) {
                // the tail from the last stage in LDS (src1 already rounded to fp16 there)
                const int kl = K > 0 ? ((K - 1) / FKC) * FKC : 0;
                const uint16_t *xt = xs + (br + r) * FLD - kl;
                const uint16_t *yt = ys + (bc + c) * FLD - kl;
                double sum = (double)res;
                for (int e = np; e < K; e++) sum += (double)(h2f_bits(xt[e]) * h2f_bits(yt[e]));
                d[(i2 * ne11 + i1) * ne01 + i0] = (float)sum;
                if (merged) merged[(i1 * ne02 + i2) * ne01 + i0] = (float)sum;
            }
        }
    }
}

// ----------------------------------------------------------------------------------- fused chains
// Back-to-back nodes of a LLaMA graph in one launch (ggml-hip-fuse.cpp defers the producer until its
// consumer arrives).  Each stage computes exactly what its own node's kernel above computes, in
// the same order, and writes that node's output too unless it shares the final output's buffer
// (in-place nodes), so every intermediate tensor holds the value ggml.c would give it.

// [sum = a + b] -> norm = sum * (1/sqrt(mean(sum^2) + eps)) -> out = norm * w  (w one row); one wave
// per row.  a == nullptr: no add (norm of x = b).  sum / norm == nullptr: not stored.
__global__ __launch_bounds__(TPB) void k_add_rms_norm_mul(const float *a, const float *b, float *sum, float *norm,
                                                          const float *w, float *out, int64_t ncols, int64_t nrows) {
    const int64_t r = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const int64_t o = r * ncols;
    double s = 0.0;
    for (int64_t i = lane; i < ncols; i += 64) {
        const float v = a ? a[o + i] + b[o + i] : b[o + i];
        if (sum) sum[o + i] = v;
        s += (double)(v * v);
    }
    s = wave_sum_d(s);
    const float mean = (float)(s / (double)ncols);
    const float scale = 1.0f / (float)__builtin_sqrt((double)(mean + 1e-6f));
    for (int64_t i = lane; i < ncols; i += 64) {
        // the same float as above (re-read from sum, which may alias a or b, written by this lane)
        const float v = sum ? sum[o + i] : (a ? a[o + i] + b[o + i] : b[o + i]);
        const float y = v * scale;
        if (norm) norm[o + i] = y;
        out[o + i] = y * w[i];
    }
}

// scaled = x * v -> masked (i > n_past + j: -inf) -> soft_max; one wave per row
__global__ __launch_bounds__(TPB) void k_scale_mask_soft_max(const float *x, float *scaled, float *masked, float *d,
                                                             float v, int64_t ncols, int64_t nrows,
                                                             int64_t rows_per_channel, int n_past, const uint16_t *table) {
    const int64_t r = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const int64_t o = r * ncols, j = r % rows_per_channel;
    auto val = [&](int64_t i) __attribute__((always_inline)) {
        const float sv = x[o + i] * v;
        return i > n_past + j ? -INFINITY : sv;
    };
    float mx = -INFINITY;
    for (int64_t i = lane; i < ncols; i += 64) mx = fmaxf(mx, val(i));
    mx = wave_max_f(mx);
    double s = 0.0;
    for (int64_t i = lane; i < ncols; i += 64) {
        const float sv = x[o + i] * v;
        const float m = i > n_past + j ? -INFINITY : sv;
        if (scaled) scaled[o + i] = sv;
        if (masked) masked[o + i] = m;
        float e = 0.0f;
        if (m != -INFINITY) {
            e = h2f_bits(lut_exp(table, f2h_bits(m - mx)));
            s += (double)e;
        }
        d[o + i] = e;
    }
    s = wave_sum_d(s);
    const float inv = (float)(1.0 / s);
    for (int64_t i = lane; i < ncols; i += 64) d[o + i] = d[o + i] * inv;
}

// The same chain with the row held in registers (ncols <= 64 * NV): x read once, d written once (the
// kernel above reads x twice and writes d twice); every value is computed by the same operations in the
// same per-lane order (max, then e and its double sum in i = lane, lane + 64, ... order, then the wave
// sums), so the output bits are the same.  Rows are independent, so d may alias x (the in-place chain).
template <int NV>
__global__ __launch_bounds__(TPB) void k_scale_mask_soft_max_reg(const float *x, float *scaled, float *masked,
                                                                 float *d, float v, int64_t ncols, int64_t nrows,
                                                                 int64_t rows_per_channel, int n_past,
                                                                 const uint16_t *table) {
    const int64_t r = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const int64_t o = r * ncols, j = r % rows_per_channel;
    float m[NV];
    // the row's loads and then its table lookups as unconditional loads of clamped indices, so each
    // group issues back to back (a load under a branch waits at the join); values selected after
    float xv[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) xv[k] = x[o + (lane + 64 * k < ncols ? lane + 64 * k : ncols - 1)];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        const int64_t i = lane + 64 * k;
        m[k] = -INFINITY;
        if (i < ncols) {
            const float sv = xv[k] * v;
            m[k] = i > n_past + j ? -INFINITY : sv;
            if (scaled) scaled[o + i] = sv;
            if (masked) masked[o + i] = m[k];
            mx = fmaxf(mx, m[k]);
        }
    }
    mx = wave_max_f(mx);
    uint16_t tv[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) tv[k] = lut_exp(table, f2h_bits(m[k] - mx));   // -inf - mx: a valid index, unused
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        float e = 0.0f;
        if (m[k] != -INFINITY) {
            e = h2f_bits(tv[k]);
            s += (double)e;
        }
        m[k] = e;
    }
    s = wave_sum_d(s);
    const float inv = (float)(1.0 / s);
#pragma unroll
    for (int k = 0; k < NV; k++) {
        const int64_t i = lane + 64 * k;
        if (i < ncols) d[o + i] = m[k] * inv;
    }
}

// Decode attention's second half: scale -> diag_mask_inf -> soft_max of each head's KQ row (one
// query row per head) and KQV = V.fp16(softmax) with its merged copy.  SM_SPLIT workgroups per head
// each recompute the row's softmax (max, the exp table, the double sum of exactly representable
// terms: order-free, so every workgroup gets the same bits as k_scale_mask_soft_max) and take
// 32 of the head's KQV outputs, 32 lanes per output as k_mul_mat_f16_f32 does.  Workgroup 0 of a
// head stores the softmax row (and scaled / masked) unless nullptr: the caller passes nullptr for a
// buffer that aliases kq (the in-place chain), which the other workgroups are still reading.
// KQ: the head's KQ row first, in LDS (the whole decode attention in one launch): key j of head i2 is
// ggml_vec_dot_f16 of K row j (f16, element stride 2 bytes) and fp16(q), the arithmetic of
// k_mul_mat_f16_f32 (lane l of 32 takes elements l + 32 m in order, the same reduction tree and double
// tail), one 32-lane group per key; workgroup 0 of the head stores it to kq_out unless nullptr.
#ifdef ATTN_STAMPS       // diagnostic builds only: per workgroup s_memrealtime at the phase boundaries
__device__ uint64_t *g_attn_stamps = nullptr;
#define ATTN_STAMP(k)                                                                                 \
    if (g_attn_stamps && threadIdx.x == 0) {                                                          \
        volatile uint64_t *st_ = g_attn_stamps + (uint64_t)blockIdx.x * 8;                            \
        st_[k] = __builtin_amdgcn_s_memrealtime();                                                    \
    }
#else
#define ATTN_STAMP(k)
#endif
struct AttnKQ {
    const char *ks;            // K view: key j of head h at ks + h * nb02k + j * nb01k
    int64_t nb01k, nb02k;
    const float *q;            // q of head h at q + h * nb02q / 4 (contiguous hd floats)
    int64_t nb02q;
    int hd;                    // head dimension, <= SM_HD
    float *kq_out;
};
// threads per decode-attention workgroup: 32 KQV outputs per 1024 threads, 512 for short rows (the head's
// outputs over twice the workgroups; tools/attn_ab.py: fused 5.5 / 6.1 vs 6.2 / 6.4 us at 40 / 72 keys, slower
// from ~130 keys on, where each workgroup's KQ phase gets longer)
constexpr int SM_PF = 16, SM_HD = 256;
constexpr int64_t ATTN_SMALL_WG_MAX_KV = 100;
#ifndef ATTN_KQ_U
#define ATTN_KQ_U 4         // keys in flight per 32-lane group in the fused KQ phase
#endif
// KQM: 0 (kq read from memory) or the K-row elements per lane, ceil(hd / 32) rounded up to 2, 4 or 8
template <int KQM, int T>
__global__ __launch_bounds__(T) void k_softmax_kqv(const float *kq, float *scaled, float *masked, float *sm,
                                                            float v, int n_past, const uint16_t *table, int64_t nkv,
                                                            const char *vs, int64_t nb01v, int64_t nb02v, int64_t nout,
                                                            int splits, float *kqv, float *merged, const AttnKQ aq) {
    extern __shared__ float row[];                     // [nkv]
    __shared__ float redf[T / 64];
    __shared__ double redd[T / 64];
    const int64_t i2 = blockIdx.x / splits;
    const int part = blockIdx.x % splits;
    const int tid = threadIdx.x, g = tid >> 5, l = tid & 31, wave = tid >> 6, lane = tid & 63;
    const int64_t o = i2 * nkv;
    const bool store = part == 0;
    ATTN_STAMP(0)
    // this lane's first SM_PF V^T values and the row's tail (K % 32 values, one per lane) are loaded
    // before the softmax, so their latency runs under it: unconditional loads of clamped (valid)
    // addresses, so they issue back to back (a load under a branch waits at the join); the products
    // below use the same values in the same order
    const int64_t r = (int64_t)part * (T / 32) + g;
    const bool live = r < nout;
    const uint16_t *xr = (const uint16_t *)(vs + i2 * nb02v + (live ? r : 0) * nb01v);
    const int K = (int)nkv;
    const int np = K & ~31, tl = K - np;
    // (measured, tools/attn_stamps.py: issued after the K row or after the KQ barrier instead, the fused
    // launch is 0.3-0.4 us longer; the row's max folded into the KQ phase saves its softmax pass but costs
    // as much in the KQ phase)
    uint16_t vpre[SM_PF];
#pragma unroll
    for (int j = 0; j < SM_PF; j++) vpre[j] = xr[min(l + 32 * j, K - 1)];
    const uint16_t vtail = xr[min(np + l, K - 1)];
    constexpr bool KQ = KQM > 0;
    if constexpr (KQ) {
        const int hd = aq.hd, hnp = hd & ~31, htl = hd - hnp, hkl = hd - 1;
        const float *qr = reinterpret_cast<const float *>(reinterpret_cast<const char *>(aq.q) + i2 * aq.nb02q);
        // q's raw values and the first KQ_U keys' K-row loads are all issued before q's fp16 conversion
        // (f2h_bits' opaque barrier waits for its operand): one memory round trip, not two
        float qv[KQM];
#pragma unroll
        for (int m = 0; m < KQM; m++) qv[m] = qr[min(l + 32 * m, hkl)];
        const float qtv = qr[min(hnp + l, hkl)];
        // KQ_U keys per group in flight: every key's K-row loads (unconditional, clamped indices) are issued
        // before the first key's products, so a group waits for one memory round trip per KQ_U keys
        constexpr int KQ_U = ATTN_KQ_U, G = T / 32;
        uint16_t kb[KQ_U][KQM], kt[KQ_U];
        auto load_keys = [&](int64_t j0) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < KQ_U; u++) {
                const int64_t jc = min(j0 + (int64_t)u * G, nkv - 1);
                const uint16_t *kr = reinterpret_cast<const uint16_t *>(aq.ks + i2 * aq.nb02k + jc * aq.nb01k);
#pragma unroll
                for (int m = 0; m < KQM; m++) kb[u][m] = kr[min(l + 32 * m, hkl)];
                kt[u] = kr[min(hnp + l, hkl)];
            }
        };
        load_keys(g);
        float qh[KQM];                                 // fp16(q) of this lane's elements
#pragma unroll
        for (int m = 0; m < KQM; m++) qh[m] = h2f_bits(f2h_bits(qv[m]));
        const float qt = h2f_bits(f2h_bits(qtv));
        for (int64_t j0 = g; j0 < nkv; j0 += KQ_U * G) {
            if (j0 != g) load_keys(j0);
#pragma unroll
            for (int u = 0; u < KQ_U; u++) {
                const int64_t j = j0 + (int64_t)u * G;
                if (j >= nkv) break;                   // uniform per 32-lane group
                float acc = 0.0f;
#pragma unroll
                for (int m = 0; m < KQM; m++)
                    if (32 * m < hnp) acc = fmaf(h2f_bits(kb[u][m]), qh[m], acc);
                const float pt = l < htl ? h2f_bits(kt[u]) * qt : 0.0f;
                const float p16 = __shfl_xor(acc, 16, 32);
                const float a = acc + p16;
                const float p8 = __shfl_xor(a, 8, 32);
                const float c = a + p8;
                const float c4 = __shfl_xor(c, 4, 32);
                const float t0 = c + c4;
                const float t01 = t0 + __shfl_xor(t0, 1, 32);
                const float t23 = __shfl(t01, 2, 32);
                const float res = t01 + t23;
                double sum = (double)res;
                for (int e = 0; e < htl; e++) sum += (double)__shfl(pt, e, 32);
                if (l == 0) {
                    row[j] = (float)sum;
                    if (store && aq.kq_out) aq.kq_out[o + j] = (float)sum;
                }
            }
        }
        __syncthreads();
    }
    ATTN_STAMP(1)
    auto kq_at = [&](int64_t i) { return KQ ? row[i] : kq[o + i]; };
    float mx = -INFINITY;
    for (int64_t i = tid; i < nkv; i += T) mx = fmaxf(mx, i > n_past ? -INFINITY : kq_at(i) * v);
    mx = wave_max_f(mx);
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = redf[0];
    for (int w = 1; w < T / 64; w++) mx = fmaxf(mx, redf[w]);
    double ssum = 0.0;
    for (int64_t i = tid; i < nkv; i += T) {
        const float sv = kq_at(i) * v;
        const float m = i > n_past ? -INFINITY : sv;
        float e = 0.0f;
        if (m != -INFINITY) {
            e = h2f_bits(lut_exp(table, f2h_bits(m - mx)));
            ssum += (double)e;
        }
        row[i] = e;
        if (store) {
            if (scaled) scaled[o + i] = sv;
            if (masked) masked[o + i] = m;
        }
    }
    ssum = wave_sum_d(ssum);
    if (lane == 0) redd[wave] = ssum;
    __syncthreads();
    ssum = 0.0;
    for (int w = 0; w < T / 64; w++) ssum += redd[w];
    const float inv = (float)(1.0 / ssum);
    for (int64_t i = tid; i < nkv; i += T) {
        const float pv = row[i] * inv;
        row[i] = pv;
        if (store && sm) sm[o + i] = pv;
    }
    __syncthreads();
    ATTN_STAMP(2)
    // KQV output r of this head: V^T row r (nkv f16) . fp16(softmax row)
    if (!live) return;
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < SM_PF; j++) {
        const int e = l + 32 * j;
        if (e < np) acc = fmaf(h2f_bits(vpre[j]), h2f_bits(f2h_bits(row[e])), acc);
    }
    for (int e0 = 32 * SM_PF; e0 < np; e0 += 32 * SM_PF) {   // longer rows: SM_PF loads per batch
        uint16_t vb[SM_PF];
#pragma unroll
        for (int j = 0; j < SM_PF; j++) vb[j] = xr[min(e0 + l + 32 * j, K - 1)];
#pragma unroll
        for (int j = 0; j < SM_PF; j++) {
            const int e = e0 + l + 32 * j;
            if (e < np) acc = fmaf(h2f_bits(vb[j]), h2f_bits(f2h_bits(row[e])), acc);
        }
    }
    const float p16 = __shfl_xor(acc, 16, 32);
    const float a = acc + p16;
    const float p8 = __shfl_xor(a, 8, 32);
    const float c = a + p8;
    const float c4 = __shfl_xor(c, 4, 32);
    const float t0 = c + c4;
    const float t01 = t0 + __shfl_xor(t0, 1, 32);
    const float t23 = __shfl(t01, 2, 32);
    const float res = t01 + t23;
    // the tail e >= np in double, in order of e (each product formed by its lane, gathered in turn)
    const float pt = l < tl ? h2f_bits(vtail) * h2f_bits(f2h_bits(row[np + l])) : 0.0f;
    double sum = (double)res;
    for (int e = 0; e < tl; e++) sum += (double)__shfl(pt, e, 32);
    if (l == 0) {
        kqv[i2 * nout + r] = (float)sum;
        if (merged) merged[i2 * nout + r] = (float)sum;
    }
    ATTN_STAMP(3)
}

// row of workgroup i for the image producers: the 8 rows of octet q = 8 * (j / 8) + i % 8 (j = i / 8)
// on XCD i % 8, consecutively
__device__ __forceinline__ int64_t x9_row(int64_t i) {
    const int64_t j = i >> 3;
    return (((j >> 3) << 3) + (i & 7)) * 8 + (j & 7);
}

// The same [add ->] rms_norm [-> mul] with one 1024-thread workgroup per row: every thread loads
// its float4 pieces of the row at once (up to NV per thread, held in registers), the double sum is
// reduced by shuffles and LDS, and the row is written from the registers.  One wave per row walks
// a 4096-wide row with 64 dependent load round trips (24 us per launch, measured); this form takes
// one.  Rows with ncols % 4 != 0, more than 4096*NV values or unaligned pointers use the kernels above.
// IMG: the k_gemm9 x image of `out` is written beside it (the q4_0 mul_mats that consume the row then
// skip k_prep9_x): thread t's pieces are elements 4t, 4t + 4096, ... of the row, so the 8 threads of a
// q8_0 block are 8 consecutive lanes, as x9_store_lane takes them, and the codes come from the very
// floats stored in out (the image is bitwise k_prep9_x's of out).  The image keeps 8 consecutive
// tokens' 16-byte pieces in one 128-byte line, so the 8 rows of a line run on one XCD (workgroup i runs
// on XCD i % 8): the line is completed in that XCD's L2 instead of leaving it as 8 partial writes
// (x9_row; the grid is nrows rounded up to 64).
constexpr int RN_THREADS = 1024, RN_NV = 4;
template <bool IMG>
__global__ __launch_bounds__(RN_THREADS) void k_row_norm4(const float *a, const float *b, float *sum, float *norm,
                                                          const float *w, float *out, int64_t ncols, int64_t nrows,
                                                          uint8_t *ximg, uint16_t *xd16, int64_t Np) {
    __shared__ double part[RN_THREADS / 64];
    const int tid = threadIdx.x;
    const int64_t row = IMG ? x9_row(blockIdx.x) : (int64_t)blockIdx.x;
    if (IMG && row >= nrows) return;                     // workgroup-uniform: rows past the padded grid
    const int64_t o = row * ncols;
    const int64_t n4 = ncols / 4;
    float4 v[RN_NV];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < RN_NV; k++) {
        const int64_t i4 = tid + (int64_t)k * RN_THREADS;
        if (i4 < n4) {
            float4 x = reinterpret_cast<const float4 *>(b + o)[i4];
            if (a) {
                const float4 y = reinterpret_cast<const float4 *>(a + o)[i4];
                x = make_float4(y.x + x.x, y.y + x.y, y.z + x.z, y.w + x.w);   // a + b, as k_add_f32
                if (sum) reinterpret_cast<float4 *>(sum + o)[i4] = x;
            }
            v[k] = x;
            s += (double)(x.x * x.x);
            s += (double)(x.y * x.y);
            s += (double)(x.z * x.z);
            s += (double)(x.w * x.w);
        }
    }
    s = wave_sum_d(s);
    if ((tid & 63) == 0) part[tid >> 6] = s;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < RN_THREADS / 64; i++) t += part[i];
    const float mean = (float)(t / (double)ncols);
    const float scale = 1.0f / (float)__builtin_sqrt((double)(mean + 1e-6f));
#pragma unroll
    for (int k = 0; k < RN_NV; k++) {
        const int64_t i4 = tid + (int64_t)k * RN_THREADS;
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i4 < n4) {
            const float4 x = v[k];
            const float4 y = make_float4(x.x * scale, x.y * scale, x.z * scale, x.w * scale);
            if (norm) reinterpret_cast<float4 *>(norm + o)[i4] = y;
            if (out) {
                const float4 g = reinterpret_cast<const float4 *>(w)[i4];
                r = make_float4(y.x * g.x, y.y * g.y, y.z * g.z, y.w * g.w);
                reinterpret_cast<float4 *>(out + o)[i4] = r;
            }
        }
        if constexpr (IMG) {
            if ((int64_t)k * RN_THREADS < n4)            // workgroup-uniform; every lane of a live wave calls
                x9_store_lane(r, tid & 7, row, i4 >> 3, i4 < n4, ximg, xd16, Np);
        }
    }
}

// Fast mode (GGML_HIP_EXACT off): the same products on the f16 matrix cores (v_mfma_f32_32x32x16_f16,
// exact fp16 products, fp32 sums in the instruction's order instead of the AVX chains', so within the
// fp32-accumulation bound of the reference rather than bitwise).  A = src1 rows rounded to fp16 (the
// tokens i1: MFMA rows), B = src0 rows as stored (i0: MFMA columns, so a row of 32 outputs is one
// coalesced store).  Workgroup = 64 tokens x 128 src0 rows of one channel, 4 waves of 32 x 64 (two MFMAs
// sharing A).  K runs in chunks of 32 staged through LDS (src1 converted to fp16 on the way in), the next
// chunk's global loads in flight while this chunk's MFMAs run (double-buffered LDS, one barrier per
// chunk): every global load is a 16/32-byte piece of a row, several lanes per row — the direct-load form
// (each lane 16-32 B of a different row per instruction, 32 rows per load instruction) ran 22-25 us per
// 500-token call, this one 15-16 (KQ) / 15 (KQV, 32-token tiles), tools/r4_ab_f16.sh.  vec: row starts 16-byte aligned (vector loads), else element loads;
// zero past K.
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16v __attribute__((ext_vector_type(16)));
// K chunk 32 (30 / 46 KB of LDS: 5 / 3 workgroups per CU); chunks of 64 measured slower (KQ 19.7 vs 15-16 us:
// 2 workgroups per CU), tools/r4_ab_f16.sh
constexpr int FM_TO = 128, FM_KC = 32;               // workgroup tile: TI tokens (i1) x 128 src0 rows (i0); K chunk
constexpr int FM_P = FM_KC + 8;                       // LDS row pitch in halves (80 B: ds_read_b128 rows staggered)

// TI = 64: 4 waves of 32 tokens x 64 rows (two MFMAs sharing A); TI = 32 (few src0 rows, e.g. KQV's 128:
// twice the workgroups): 4 waves of 32 tokens x 32 rows
template <int TI>
__global__ __launch_bounds__(TPB) void k_mul_mat_f16_f32_mfma(const char *s0, const char *s1, float *d, int K,
                                                              int64_t ne01, int64_t ne11, int64_t ne02, int64_t nb01,
                                                              int64_t nb02, int64_t nb11, int64_t nb12, float *merged,
                                                              int vec) {
    constexpr int AV = TI * FM_KC / TPB;              // src1 floats staged per thread (8 or 4)
    static_assert(AV % 4 == 0 && FM_KC % AV == 0, "src1 staging in float4 pieces");
    constexpr int BV = FM_TO * FM_KC / TPB;           // src0 halves staged per thread (32)
    __shared__ __attribute__((aligned(16))) _Float16 as[2][TI * FM_P];
    __shared__ __attribute__((aligned(16))) _Float16 bs[2][FM_TO * FM_P];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int rl = lane & 31, kh = lane >> 5;
    const int64_t i2 = blockIdx.z;
    const int64_t T0 = (int64_t)blockIdx.y * TI, O0 = (int64_t)blockIdx.x * FM_TO;
    // staging roles: src1 row ra (AV values from ka), src0 row rb (BV halves from kb); rows past the matrix
    // are clamped (loaded, never stored)
    const int ra = t / (FM_KC / AV), ka = (t % (FM_KC / AV)) * AV, rb = t / (FM_KC / BV), kb = (t % (FM_KC / BV)) * BV;
    const int64_t ga = T0 + ra < ne11 ? T0 + ra : ne11 - 1, gb = O0 + rb < ne01 ? O0 + rb : ne01 - 1;
    const float *ya = (const float *)(s1 + i2 * nb12 + ga * nb11);
    const _Float16 *xb = (const _Float16 *)(s0 + i2 * nb02 + gb * nb01);
    struct Stage {
        float4 y[AV / 4];
        h16x8 x[BV / 8];
    };
    auto gload = [&](int k0, Stage &g) __attribute__((always_inline)) {
        const int k = k0 + ka, kx = k0 + kb;
#pragma unroll
        for (int q = 0; q < AV / 4; q++) {
            const int kq = k + 4 * q;
            if (vec && kq + 4 <= K) {
                g.y[q] = *reinterpret_cast<const float4 *>(ya + kq);
            } else {
                g.y[q] = make_float4(kq < K ? ya[kq] : 0.0f, kq + 1 < K ? ya[kq + 1] : 0.0f, kq + 2 < K ? ya[kq + 2] : 0.0f,
                                     kq + 3 < K ? ya[kq + 3] : 0.0f);
            }
        }
#pragma unroll
        for (int q = 0; q < BV / 8; q++) {
            const int kq = kx + 8 * q;
            if (vec && kq + 8 <= K) {
                g.x[q] = *reinterpret_cast<const h16x8 *>(xb + kq);
            } else {
#pragma unroll
                for (int e = 0; e < 8; e++) g.x[q][e] = kq + e < K ? xb[kq + e] : (_Float16)0.0f;
            }
        }
    };
    typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
    auto lstore = [&](int buf, const Stage &g) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < AV / 4; q++) {            // 4 values (8 bytes) per float4 piece
            const float4 u = g.y[q];
            const h16x4 a = {(_Float16)u.x, (_Float16)u.y, (_Float16)u.z, (_Float16)u.w};
            *reinterpret_cast<h16x4 *>(&as[buf][ra * FM_P + ka + 4 * q]) = a;
        }
#pragma unroll
        for (int q = 0; q < BV / 8; q++) *reinterpret_cast<h16x8 *>(&bs[buf][rb * FM_P + kb + 8 * q]) = g.x[q];
    };
    // this lane's A row and B rows (TI = 64: wave = token half x row half, B rows bt and bt + 32; TI = 32:
    // wave = row quarter, B row bt)
    const int at = TI == 64 ? 32 * (wave & 1) + rl : rl;
    const int bt = TI == 64 ? 64 * (wave >> 1) + rl : 32 * wave + rl;
    f32x16v acc0 = {}, acc1 = {};
    Stage g;
    gload(0, g);
    lstore(0, g);
    __syncthreads();
    const int nc = (K + FM_KC - 1) / FM_KC;
    for (int c = 0; c < nc; c++) {
        const int buf = c & 1;
        if (c + 1 < nc) gload((c + 1) * FM_KC, g);
#pragma unroll
        for (int st = 0; st < FM_KC / 16; st++) {
            const int ko = 16 * st + 8 * kh;
            const h16x8 a = *reinterpret_cast<const h16x8 *>(&as[buf][at * FM_P + ko]);
            const h16x8 b0 = *reinterpret_cast<const h16x8 *>(&bs[buf][bt * FM_P + ko]);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b0, acc0, 0, 0, 0);
            if constexpr (TI == 64) {
                const h16x8 b1 = *reinterpret_cast<const h16x8 *>(&bs[buf][(bt + 32) * FM_P + ko]);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b1, acc1, 0, 0, 0);
            }
        }
        if (c + 1 < nc) lstore(buf ^ 1, g);
        __syncthreads();
    }
    // acc[r] = D[token t0 + (r & 3) + 8 (r >> 2) + 4 kh][src0 row o0 (+ 32) + rl]
    const int64_t t0 = T0 + (TI == 64 ? 32 * (wave & 1) : 0), o0 = O0 + (TI == 64 ? 64 * (wave >> 1) : 32 * wave);
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int64_t i1 = t0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        if (i1 >= ne11) continue;
#pragma unroll
        for (int h = 0; h < (TI == 64 ? 2 : 1); h++) {
            const int64_t i0 = o0 + 32 * h + rl;
            if (i0 >= ne01) continue;
            const float v = h ? acc1[r] : acc0[r];
            d[(i2 * ne11 + i1) * ne01 + i0] = v;
            if (merged) merged[(i1 * ne02 + i2) * ne01 + i0] = v;
        }
    }
}

// u = silu(a) (fp16 table) -> out = u * b
__global__ __launch_bounds__(TPB) void k_silu_mul(const float *a, const float *b, float *u, float *out, int64_t n,
                                                  const uint16_t *table) {
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const float s = h2f_bits(lut_silu(table, f2h_bits(a[i])));
    if (u) u[i] = s;
    out[i] = s * b[i];
}

// k_silu_mul on float4 pieces of rows of ncols (ncols % 64 == 0) with the k_gemm9 x image of out written
// beside it (bitwise k_prep9_x's of out); c4 = ncols / 4, so a q8_0 block is 8 consecutive lanes.  A
// workgroup takes chunk c of TPB float4s of one row; the same chunk of 8 consecutive rows runs on one
// XCD (as k_row_norm4<true>): workgroup i -> XCD x = i % 8, its j = i / 8-th item there = (row t = j % 8
// of octet 8 * ((j / 8) / C) + x, chunk (j / 8) % C), C = chunks per row.
__global__ __launch_bounds__(TPB) void k_silu_mul_x9(const float *a, const float *b, float *u, float *out, int64_t nrows,
                                                     int64_t c4, int64_t C, const uint16_t *table, uint8_t *ximg,
                                                     uint16_t *xd16, int64_t Np) {
    const int64_t i = blockIdx.x, j = i >> 3, rest = j >> 3;
    const int64_t row = ((rest / C) * 8 + (i & 7)) * 8 + (j & 7), chunk = rest % C;
    if (row >= nrows) return;                            // workgroup-uniform
    const int64_t c = chunk * TPB + threadIdx.x;         // float4 index within the row
    const bool in = c < c4;
    const int64_t i4 = row * c4 + c;
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (in) {
        const float4 av = reinterpret_cast<const float4 *>(a)[i4], bv = reinterpret_cast<const float4 *>(b)[i4];
        // the four table indices first, then the four lookups back to back (interleaved with the
        // conversions they were issued and waited for one at a time)
        const uint16_t h0 = f2h_bits(av.x), h1 = f2h_bits(av.y), h2 = f2h_bits(av.z), h3 = f2h_bits(av.w);
        const uint16_t t0 = lut_silu(table, h0), t1 = lut_silu(table, h1), t2 = lut_silu(table, h2), t3 = lut_silu(table, h3);
        const float4 sv = make_float4(h2f_bits(t0), h2f_bits(t1), h2f_bits(t2), h2f_bits(t3));
        if (u) reinterpret_cast<float4 *>(u)[i4] = sv;
        r = make_float4(sv.x * bv.x, sv.y * bv.y, sv.z * bv.z, sv.w * bv.w);
        reinterpret_cast<float4 *>(out)[i4] = r;
    }
    x9_store_lane(r, threadIdx.x & 7, row, c >> 3, in, ximg, xd16, Np);
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }   // nullptr passes (not accessed)

bool row_norm4_ok(int64_t ncols, const void *a, const void *b, const void *sum, const void *norm, const void *w,
                  const void *out) {
    return ncols % 4 == 0 && ncols <= 4 * RN_THREADS * RN_NV && al16(a) && al16(b) && al16(sum) && al16(norm) &&
           al16(w) && al16(out);
}

}  // namespace

hipError_t op_add_rms_norm_mul_f32(const float *a, const float *b, float *sum, float *norm, const float *w, float *out,
                                   int64_t ncols, int64_t nrows, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    if (row_norm4_ok(ncols, a, b, sum, norm, w, out))
        launch_k(k_row_norm4<false>, dim3((unsigned)nrows), dim3(RN_THREADS), 0, s, a, b, sum, norm, w, out, ncols,
                 (int64_t)0, (uint8_t *)nullptr, (uint16_t *)nullptr, (int64_t)0);
    else
        launch_k(k_add_rms_norm_mul, dim3(blocks(nrows, TPB / 64)), dim3(TPB), 0, s, a, b, sum, norm, w, out,
                           ncols, nrows);
    return hipGetLastError();
}

bool op_x9_ok(int64_t ncols, int64_t nrows) {
    return nrows > 0 && ncols > 0 && ncols % 64 == 0 && ncols <= 4 * RN_THREADS * RN_NV && nrows < (1 << 30);
}

hipError_t op_add_rms_norm_mul_f32_x9(const float *a, const float *b, float *sum, float *norm, const float *w, float *out,
                                      int64_t ncols, int64_t nrows, void *xws, int64_t Np, hipStream_t s) {
    if (!op_x9_ok(ncols, nrows) || !out || !xws || Np < nrows || !x9_fits(ncols, Np) || !row_norm4_ok(ncols, a, b, sum, norm, w, out))
        return hipErrorInvalidValue;
    uint8_t *ximg = (uint8_t *)xws;
    uint16_t *xd16 = (uint16_t *)((char *)xws + (size_t)(ncols / 32) * Np * 48);
    launch_k(k_row_norm4<true>, dim3((unsigned)((nrows + 63) & ~63)), dim3(RN_THREADS), 0, s, a, b, sum, norm, w, out,
             ncols, nrows, ximg, xd16, Np);
    return hipGetLastError();
}

hipError_t op_silu_mul_f32_x9(const float *a, const float *b, float *u, float *out, int64_t ncols, int64_t nrows,
                              const uint16_t *table, void *xws, int64_t Np, hipStream_t s) {
    if (!op_x9_ok(ncols, nrows) || !out || !xws || Np < nrows || !x9_fits(ncols, Np) || !al16(a) || !al16(b) || !al16(u) || !al16(out))
        return hipErrorInvalidValue;
    uint8_t *ximg = (uint8_t *)xws;
    uint16_t *xd16 = (uint16_t *)((char *)xws + (size_t)(ncols / 32) * Np * 48);
    const int64_t c4 = ncols / 4, C = (c4 + TPB - 1) / TPB;
    launch_k(k_silu_mul_x9, dim3((unsigned)(((nrows + 63) & ~63) * C)), dim3(TPB), 0, s, a, b, u, out, nrows, c4, C, table,
             ximg, xd16, Np);
    return hipGetLastError();
}

hipError_t op_scale_mask_soft_max_f32(const float *x, float *scaled, float *masked, float *d, float v, int64_t ncols,
                                      int64_t nrows, int64_t rows_per_channel, int n_past, const uint16_t *table,
                                      hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    const dim3 g(blocks(nrows, TPB / 64));
    // the row in registers where it fits (prefill KQ rows up to 2048 keys), else two passes over memory
    if (ncols <= 64 * 8)
        launch_k(k_scale_mask_soft_max_reg<8>, g, dim3(TPB), 0, s, x, scaled, masked, d, v, ncols, nrows, rows_per_channel,
                 n_past, table);
    else if (ncols <= 64 * 32)
        launch_k(k_scale_mask_soft_max_reg<32>, g, dim3(TPB), 0, s, x, scaled, masked, d, v, ncols, nrows,
                 rows_per_channel, n_past, table);
    else
        launch_k(k_scale_mask_soft_max, g, dim3(TPB), 0, s, x, scaled, masked, d, v, ncols, nrows, rows_per_channel,
                 n_past, table);
    return hipGetLastError();
}

template <int KQM, int T>
static void launch_softmax_kqv(const float *kq, float *scaled, float *masked, float *sm, float v, int n_past,
                               const uint16_t *table, int64_t nkv, int64_t nhead, const void *vs, int64_t nb01v,
                               int64_t nb02v, int64_t nout, float *kqv, float *merged, const AttnKQ &aq, hipStream_t s) {
    const int splits = (int)((nout + T / 32 - 1) / (T / 32));
    launch_k(k_softmax_kqv<KQM, T>, dim3((unsigned)(nhead * splits)), dim3(T), (size_t)nkv * 4, s, kq, scaled, masked, sm,
             v, n_past, table, nkv, (const char *)vs, nb01v, nb02v, nout, splits, kqv, merged, aq);
}

hipError_t op_softmax_kqv(const float *kq, float *scaled, float *masked, float *sm, float v, int n_past,
                          const uint16_t *table, int64_t nkv, int64_t nhead, const void *vs, int64_t nb01v, int64_t nb02v,
                          int64_t nout, float *kqv, float *merged, hipStream_t s) {
    if (nhead <= 0 || nkv <= 0 || nout <= 0) return hipSuccess;
    if (nkv <= ATTN_SMALL_WG_MAX_KV)
        launch_softmax_kqv<0, 512>(kq, scaled, masked, sm, v, n_past, table, nkv, nhead, vs, nb01v, nb02v, nout, kqv,
                                   merged, AttnKQ{}, s);
    else
        launch_softmax_kqv<0, 1024>(kq, scaled, masked, sm, v, n_past, table, nkv, nhead, vs, nb01v, nb02v, nout, kqv,
                                    merged, AttnKQ{}, s);
    return hipGetLastError();
}

#ifdef ATTN_STAMPS
extern "C" int ggml_hip_debug_attn_stamps(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t op_kq_softmax_kqv(const void *ks, int64_t nb01k, int64_t nb02k, const float *q, int64_t nb02q, int hd,
                             float *kq, float *scaled, float *masked, float *sm, float v, int n_past, const uint16_t *table,
                             int64_t nkv, int64_t nhead, const void *vs, int64_t nb01v, int64_t nb02v, int64_t nout,
                             float *kqv, float *merged, hipStream_t s) {
    if (nhead <= 0 || nkv <= 0 || nout <= 0) return hipSuccess;
    if (hd < 1 || hd > SM_HD) return hipErrorInvalidValue;
    const AttnKQ aq{(const char *)ks, nb01k, nb02k, q, nb02q, hd, kq};
    const bool small = nkv <= ATTN_SMALL_WG_MAX_KV;
#define ATTN_FUSED(M)                                                                                           \
    do {                                                                                                        \
        if (small)                                                                                              \
            launch_softmax_kqv<M, 512>(nullptr, scaled, masked, sm, v, n_past, table, nkv, nhead, vs, nb01v, nb02v, \
                                       nout, kqv, merged, aq, s);                                               \
        else                                                                                                    \
            launch_softmax_kqv<M, 1024>(nullptr, scaled, masked, sm, v, n_past, table, nkv, nhead, vs, nb01v,     \
                                        nb02v, nout, kqv, merged, aq, s);                                       \
    } while (0)
    if (hd <= 64)
        ATTN_FUSED(2);
    else if (hd <= 128)
        ATTN_FUSED(4);
    else
        ATTN_FUSED(8);
#undef ATTN_FUSED
    return hipGetLastError();
}

// every finite fp16 input: the direct evaluation against the host-built table (bad[0] silu, bad[1] exp)
__global__ __launch_bounds__(TPB) void k_lut_check(const uint16_t *silu, const uint16_t *ex, int *bad) {
    const uint32_t i = blockIdx.x * TPB + threadIdx.x;
    if (i >= 65536u || (i & 0x7C00u) == 0x7C00u) return;
    if (silu_direct(i) != silu[i]) atomicAdd(bad, 1);
    if (exp_direct(i) != ex[i]) atomicAdd(bad + 1, 1);
}

hipError_t op_lut_check(const uint16_t *silu, const uint16_t *ex, int *bad_dev, hipStream_t s) {
    (void)hipGetLastError();
    launch_k(k_lut_check, dim3(65536 / TPB), dim3(TPB), 0, s, silu, ex, bad_dev);
    return hipGetLastError();
}

hipError_t op_silu_mul_f32(const float *a, const float *b, float *u, float *out, int64_t n, const uint16_t *table,
                           hipStream_t s) {
    if (n <= 0) return hipSuccess;
    launch_k(k_silu_mul, dim3(blocks(n)), dim3(TPB), 0, s, a, b, u, out, n, table);
    return hipGetLastError();
}

hipError_t op_add_f32(const float *a, const float *b, float *d, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    launch_k(k_add_f32, dim3(blocks(n)), dim3(TPB), 0, s, a, b, d, n);
    return hipGetLastError();
}

hipError_t op_mul_f32(const float *a, const float *b, float *d, int64_t ne00, int64_t ne01, int64_t ne02, int64_t ne03,
                      int64_t ne11, int64_t ne12, int64_t ne13, hipStream_t s) {
    const int64_t nrows = ne01 * ne02 * ne03;
    if (nrows * ne00 <= 0) return hipSuccess;
    launch_k(k_mul_f32, dim3(blocks(nrows * ne00)), dim3(TPB), 0, s, a, b, d, ne00, ne01, ne02, nrows, ne11,
                       ne12, ne13);
    return hipGetLastError();
}

hipError_t op_silu_f32(const float *x, float *d, int64_t n, const uint16_t *table, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    launch_k(k_silu_f32, dim3(blocks(n)), dim3(TPB), 0, s, x, d, n, table);
    return hipGetLastError();
}

hipError_t op_scale_f32(const float *x, float *d, float v, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    launch_k(k_scale_f32, dim3(blocks(n)), dim3(TPB), 0, s, x, d, v, n);
    return hipGetLastError();
}

hipError_t op_diag_mask_inf_f32(const float *x, float *d, int64_t ncols, int64_t nrows, int64_t rows_per_channel,
                                int n_past, hipStream_t s) {
    const int64_t n = ncols * nrows;
    if (n <= 0) return hipSuccess;
    launch_k(k_diag_mask_inf_f32, dim3(blocks(n)), dim3(TPB), 0, s, x, d, ncols, n, rows_per_channel, n_past);
    return hipGetLastError();
}

hipError_t op_rms_norm_f32(const float *x, float *d, int64_t ncols, int64_t nrows, int64_t ldx, int64_t ldd,
                           hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    if (ldx == ncols && ldd == ncols && row_norm4_ok(ncols, nullptr, x, nullptr, d, nullptr, nullptr))
        launch_k(k_row_norm4<false>, dim3((unsigned)nrows), dim3(RN_THREADS), 0, s, nullptr, x, nullptr, d, nullptr,
                 nullptr, ncols, (int64_t)0, (uint8_t *)nullptr, (uint16_t *)nullptr, (int64_t)0);
    else
        launch_k(k_rms_norm_f32, dim3(blocks(nrows, TPB / 64)), dim3(TPB), 0, s, x, d, ncols, nrows, ldx, ldd);
    return hipGetLastError();
}

hipError_t op_soft_max_f32(const float *x, float *d, int64_t ncols, int64_t nrows, const uint16_t *table, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    launch_k(k_soft_max_f32, dim3(blocks(nrows, TPB / 64)), dim3(TPB), 0, s, x, d, ncols, nrows, table);
    return hipGetLastError();
}

hipError_t op_rope_f32(const void *x, void *d, const int64_t ne[4], const int64_t nbx[4], const int64_t nbd[4],
                       const void *cs, int npairs, hipStream_t s) {
    const int64_t n = ne[0] / 2 * ne[1] * ne[2] * ne[3];
    if (n <= 0) return hipSuccess;
    launch_k(k_rope_f32, dim3(blocks(n)), dim3(TPB), 0, s, (const char *)x, (char *)d, ne[0], ne[1], ne[2],
                       nbx[1], nbx[2], nbx[3], nbd[1], nbd[2], nbd[3], n, (const float2 *)cs, npairs);
    return hipGetLastError();
}

hipError_t op_rope_cpy_f32(const void *x, void *d, const int64_t ne[4], const int64_t nbx[4], const int64_t nbd[4],
                           const void *cs, int npairs, void *c, bool to_f16, int64_t ne10, int64_t ne11, int64_t nb10,
                           int64_t nb11, int64_t nb12, hipStream_t s) {
    const int64_t n = ne[0] / 2 * ne[1] * ne[2] * ne[3];
    if (n <= 0) return hipSuccess;
    if (to_f16)
        launch_k(k_rope_cpy<true>, dim3(blocks(n)), dim3(TPB), 0, s, (const char *)x, (char *)d, ne[0], ne[1],
                           ne[2], nbx[1], nbx[2], nbx[3], nbd[1], nbd[2], nbd[3], n, (const float2 *)cs, npairs, (char *)c,
                           ne10, ne11, nb10, nb11, nb12);
    else
        launch_k(k_rope_cpy<false>, dim3(blocks(n)), dim3(TPB), 0, s, (const char *)x, (char *)d, ne[0], ne[1],
                           ne[2], nbx[1], nbx[2], nbx[3], nbd[1], nbd[2], nbd[3], n, (const float2 *)cs, npairs, (char *)c,
                           ne10, ne11, nb10, nb11, nb12);
    return hipGetLastError();
}

// a kind-1 copy that takes the tiled path: 2-d, the source contiguous along dim 1 and strided along
// dim 0, the target the same shape and contiguous along dim 0, at least 64 along dim 0 (prefill)
static bool elem_cpy_transposed(const ElemOp &op) {
    const int64_t es = op.f16 ? 2 : 4;
    return op.n == op.ne0 * op.ne1 && op.ne0 >= 64 && op.ne1 >= 1 && op.nbx2 == 4 && op.nbx1 != 4 &&
           op.ne10 == op.ne0 && op.ne11 == op.ne1 && op.nb10 == es;
}

static bool a_of(const void *p, int64_t a) { return ((uintptr_t)p % (uintptr_t)a) == 0; }
// a kind-0 rope that takes the two-pairs-per-thread path: every row of x and d and the (cos, sin)
// rows 16-byte aligned, an even number of pairs per row
static bool elem_rope_vec(const ElemOp &op) {
    return op.ne0 % 4 == 0 && op.npairs % 2 == 0 && a_of(op.x, 16) &&
           a_of(op.d, 16) && a_of(op.cs, 16) && op.nbx1 % 16 == 0 && op.nbx2 % 16 == 0 && op.nbx3 % 16 == 0 &&
           op.nbd1 % 16 == 0 && op.nbd2 % 16 == 0 && op.nbd3 % 16 == 0;
}

hipError_t op_cpy_f32(const void *x, void *d, bool to_f16, int64_t n, int64_t ne00, int64_t ne01, int64_t nb00,
                      int64_t nb01, int64_t nb02, int64_t ne10, int64_t ne11, int64_t nb10, int64_t nb11, int64_t nb12,
                      hipStream_t s) {
    if (n <= 0) return hipSuccess;
    ElemBatch b{};
    ElemOp &op = b.op[0];
    op.kind = 1, op.f16 = to_f16, op.x = (const char *)x, op.c = (char *)d, op.n = n;
    op.ne0 = ne00, op.ne1 = ne01, op.nbx1 = nb00, op.nbx2 = nb01, op.nbx3 = nb02;
    op.ne10 = ne10, op.ne11 = ne11, op.nb10 = nb10, op.nb11 = nb11, op.nb12 = nb12;
    if (elem_cpy_transposed(op)) {      // the transposed V-cache store: the tiled path of k_elem_batch
        b.nops = 1;
        return op_elem_batch(b, s);
    }
    if (to_f16)
        launch_k(k_cpy_f32<true>, dim3(blocks(n)), dim3(TPB), 0, s, (const char *)x, (char *)d, n, ne00, ne01,
                           nb00, nb01, nb02, ne10, ne11, nb10, nb11, nb12);
    else
        launch_k(k_cpy_f32<false>, dim3(blocks(n)), dim3(TPB), 0, s, (const char *)x, (char *)d, n, ne00, ne01,
                           nb00, nb01, nb02, ne10, ne11, nb10, nb11, nb12);
    return hipGetLastError();
}

hipError_t op_elem_batch(const ElemBatch &b, hipStream_t s) {
    if (b.nops < 1 || b.nops > ELEM_MAX) return hipErrorInvalidValue;
    ElemBatch bb = b;
    unsigned total = 0;
    for (int q = 0; q < bb.nops; q++) {
        ElemOp &op = bb.op[q];
        if (op.kind == 1 && elem_cpy_transposed(op)) {
            op.kind = 2;
            op.n = ((op.ne0 + 63) / 64) * ((op.ne1 + 63) / 64) * TPB;   // one workgroup per tile
        } else if (op.kind == 0 && elem_rope_vec(op)) {
            op.kind = 3;
            op.n /= 2;                                                     // two pairs per item
            const int64_t es = op.f16 ? 2 : 4;
            op.pack = op.c && op.ne10 % 4 == 0 && op.nb10 == es && a_of(op.c, 4 * es) && op.nb11 % (4 * es) == 0 &&
                      op.nb12 % (4 * es) == 0;
        }
        bb.block_begin[q] = total;
        total += blocks(op.n);
    }
    for (int q = bb.nops; q < ELEM_MAX; q++) bb.block_begin[q] = total;
    if (total == 0) return hipSuccess;
    // 32-bit element indices when every index and product of extents the kernel forms fits
    bool small = (uint64_t)total * TPB < (1ull << 31);
    for (int q = 0; q < bb.nops; q++) {
        const ElemOp &op = bb.op[q];
        const int64_t lim = (int64_t)1 << 31;
        small = small && op.n < lim && op.ne0 * op.ne1 < lim && op.ne0 * op.ne1 * (op.ne2 > 1 ? op.ne2 : 1) < lim &&
                op.ne10 * op.ne11 < lim && (op.kind != 0 || op.ne0 / 2 * op.ne1 * op.ne2 < lim);
    }
    if (small)
        launch_k(k_elem_batch<uint32_t>, dim3(total), dim3(TPB), 0, s, bb);
    else
        launch_k(k_elem_batch<int64_t>, dim3(total), dim3(TPB), 0, s, bb);
    return hipGetLastError();
}

hipError_t op_mul_mat_f16_f32(const void *s0, const void *s1, float *d, int K, int64_t ne01, int64_t ne11, int64_t ne02,
                              int64_t nb01, int64_t nb02, int64_t nb11, int64_t nb12, hipStream_t s, float *merged,
                              int tiled) {
    const int64_t nout = ne01 * ne11 * ne02;
    if (nout <= 0) return hipSuccess;
    static const int tiled_min = getenv("GGML_HIP_F16_TILED_MIN") ? atoi(getenv("GGML_HIP_F16_TILED_MIN")) : 8;
    static const int mfma_min = getenv("GGML_HIP_F16_MFMA_MIN") ? atoi(getenv("GGML_HIP_F16_MFMA_MIN")) : 32;
    const bool fits = ne02 <= 65535 && (ne11 + FT - 1) / FT <= 65535;
    if (fits && (tiled == 2 || (tiled == -2 && mfma_min > 0 && ne11 >= mfma_min))) {
        // fast mode, many src1 rows (prefill): the matrix cores
        auto a16 = [](int64_t v) { return (v & 15) == 0; };
        const int vec = a16((int64_t)(uintptr_t)s0) && a16(nb01) && a16(nb02) && a16((int64_t)(uintptr_t)s1) && a16(nb11) &&
                        a16(nb12);
        // few src0 rows (KQV: 128 per head): 32-token tiles, twice the workgroups
        if (ne01 <= FM_TO)
            launch_k(k_mul_mat_f16_f32_mfma<32>, dim3((unsigned)((ne01 + FM_TO - 1) / FM_TO), (unsigned)((ne11 + 31) / 32),
                                                     (unsigned)ne02),
                     dim3(TPB), 0, s, (const char *)s0, (const char *)s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12,
                     merged, vec);
        else
            launch_k(k_mul_mat_f16_f32_mfma<64>, dim3((unsigned)((ne01 + FM_TO - 1) / FM_TO), (unsigned)((ne11 + 63) / 64),
                                                     (unsigned)ne02),
                     dim3(TPB), 0, s, (const char *)s0, (const char *)s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12,
                     merged, vec);
        return hipGetLastError();
    }
    if (tiled == -2) tiled = -1;
    if (fits && (tiled > 0 || (tiled < 0 && tiled_min > 0 && ne11 >= tiled_min))) {
        // many src1 rows (prefill): tiled through LDS, same bits
        launch_k(k_mul_mat_f16_f32_tiled, dim3((unsigned)((ne01 + FT - 1) / FT), (unsigned)((ne11 + FT - 1) / FT),
                                                         (unsigned)ne02),
                           dim3(TPB), 0, s, (const char *)s0, (const char *)s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11,
                           nb12, merged);
        return hipGetLastError();
    }
    launch_k(k_mul_mat_f16_f32, dim3(blocks(nout * 32)), dim3(TPB), 0, s, (const char *)s0, (const char *)s1, d,
                       K, ne01, ne11, ne02, nb01, nb02, nb11, nb12, merged);
    return hipGetLastError();
}

}  // namespace ghip
