// q4_0_kernels.hip — hand-written gfx950 (CDNA4) kernels for the ggml q4_0 x f32 mul_mat.
//
// What each kernel restates (reference = ggml.c of Fcucgvhhhvjv/llama.cpp-q_4_0):
//   k_quantize_q8_0   quantize_row_q8_0, AVX2 branch ggml.c:1192-1275 (bit-exact: max|x|,
//                     d = amax/127.f (IEEE div), fp16(d) RNE, id = amax ? 127.f/amax : 0,
//                     q = sat8(round-half-even(x*id)))
//   k_quantize_q4_0   quantize_row_q4_0_reference ggml.c:918-953 (bit-exact)
//   k_dequantize_q4_0 dequantize_row_q4_0 ggml.c:1500-1518
//   k_gemv_q4_0<NT>   mul_mat_q_f32 (ggml.c:11353-11411) for N <= 8 tokens: INIT (q8_0 of x)
//                     fused into the prologue (into LDS, once per workgroup), COMPUTE =
//                     ggml_vec_dot_q4_0_q8_0 (ggml.c:2339-2607) with one wave64 per weight row
//   k_gemm_q4_0       the same product for prefill batches on the int8 matrix cores
//                     (v_mfma_i32_32x32x32_i8: K=32 = exactly one q4_0/q8_0 block, so every
//                     MFMA yields the exact per-block integer sum the CPU computes); k_gemm7 reads
//                     the q4_0 bytes in place, k_gemm8 an int8 image of the weights
//   k_gemm9_q4_0      the default prefill GEMM on weight images: the same exact block sums from the
//                     block-scaled fp6 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 operands), as f32
//   k_mm_exact_q4_0   exact mode: the AVX2 branch's fp32 schedule, bit for bit
//
// Numerics: every per-block integer sum is exact (as on the CPU); the fp32 accumulation of
// d_w*d_x*sumi runs in a different order than AVX2's 8-lane fma chain, so y agrees with the
// reference within the fp32-accumulation bound (tests/parity.py), not bitwise.
#include "q4_0_kernels.h"
#include "launch.h"

#include <climits>
#include <cstdlib>

namespace ghip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

static constexpr int QK = 32;
static constexpr int Q4B = 18;   // sizeof(block_q4_0)
static constexpr int Q8B = 34;   // sizeof(block_q8_0)
static constexpr int RSRC_FLAGS = 0x00020000;  // gfx950 buffer descriptor dword3 (raw, 32-bit)

__device__ __forceinline__ float h2f(uint32_t bits) {
    _Float16 h;
    const uint16_t b = (uint16_t)bits;
    __builtin_memcpy(&h, &b, 2);
    return (float)h;                       // v_cvt_f32_f16, exact
}

__device__ __forceinline__ uint32_t f2h(float f) {
    // opaque barrier: keeps hipcc from folding a preceding multiply into v_fma_mix with a +0
    // addend, which turns -0.0 into +0.0 (ggml stores fp16(-0.0) = 0x8000 for all-zero blocks)
    asm volatile("" : "+v"(f));
    const _Float16 h = (_Float16)f;        // v_cvt_f16_f32, round-to-nearest-even
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
}

// _mm256_round_ps(nearest-even) -> cvtps_epi32 (NaN / out of range -> INT_MIN) -> packs x2
__device__ __forceinline__ int q8_round_sat(float v) {
    const float r = __builtin_rintf(v);
    int i = (r >= -2147483648.0f && r < 2147483648.0f) ? (int)r : INT_MIN;
    i = i > 127 ? 127 : i;
    return i < -128 ? -128 : i;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, RSRC_FLAGS);
}

// ---- cross-lane reductions on DPP (no LDS round trip) -------------------------------------
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {      // lanes outside ROW_MASK read 0
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_QUAD_XOR1 = 0xB1;     // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;     // quad_perm [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_MIRROR = 0x140;
constexpr int DPP_ROW_BCAST15 = 0x142;
constexpr int DPP_ROW_BCAST31 = 0x143;

// max / sum over each group of 8 consecutive lanes (every lane of the group gets the result)
__device__ __forceinline__ float group8_max(float v) {
    v = fmaxf(v, dpp_f<DPP_QUAD_XOR1>(v));
    v = fmaxf(v, dpp_f<DPP_QUAD_XOR2>(v));
    return fmaxf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
}
__device__ __forceinline__ int group8_sum(int v) {
    v += dpp_i<DPP_QUAD_XOR1>(v);
    v += dpp_i<DPP_QUAD_XOR2>(v);
    return v + dpp_i<DPP_ROW_HALF_MIRROR>(v);
}
// sum over the 64 lanes; the total is valid in lane 63 (fixed order -> deterministic)
__device__ __forceinline__ float wave_sum_lane63(float v) {
    v += dpp_f<DPP_QUAD_XOR1>(v);
    v += dpp_f<DPP_QUAD_XOR2>(v);
    v += dpp_f<DPP_ROW_HALF_MIRROR>(v);
    v += dpp_f<DPP_ROW_MIRROR>(v);
    v += dpp_f<DPP_ROW_BCAST15, 0xA>(v);
    v += dpp_f<DPP_ROW_BCAST31, 0xC>(v);
    return v;
}

// One q8_0 block spread over 8 consecutive lanes, 4 floats each (lane group g = lane>>3).
// Returns the packed int8x4 of this lane; d16 = fp16(amax/127.f); qsum = sum of the 32 q.
__device__ __forceinline__ uint32_t q8_block_lane(float4 v, uint32_t &d16, int &qsum) {
    float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    a = group8_max(a);
    const float d = a / 127.f;                         // correctly rounded (no fast-math)
    const float id = (a != 0.0f) ? 127.f / a : 0.0f;
    d16 = f2h(d);
    const int q0 = q8_round_sat(v.x * id), q1 = q8_round_sat(v.y * id);
    const int q2 = q8_round_sat(v.z * id), q3 = q8_round_sat(v.w * id);
    qsum = group8_sum(q0 + q1 + q2 + q3);
    return (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
           ((uint32_t)(q3 & 0xFF) << 24);
}

// ---------------------------------------------------------------------------------------------
// A5: q8_0 activation quantizer.  One lane per 4 floats, 8 lanes per block.

template <bool AOS>
__global__ __launch_bounds__(256) void k_quantize_q8_0(const float *__restrict__ x, int64_t K, int64_t total8,
                                                         uint8_t *__restrict__ aos, int8_t *__restrict__ qs,
                                                         float *__restrict__ dout, uint16_t *__restrict__ d16out,
                                                         int64_t N) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total8) return;                           // total8 % 8 == 0: whole groups exit together
    const int64_t blk = t >> 3;                        // global block index = n*nb + b
    const int sub = (int)(t & 7);
    const float4 v = *reinterpret_cast<const float4 *>(x + t * 4);   // x[n][32b + 4sub]
    uint32_t d16;
    int qsum;
    const uint32_t packed = q8_block_lane(v, d16, qsum);
    if (AOS) {
        uint8_t *o = aos + blk * Q8B;
        uint16_t *o16 = reinterpret_cast<uint16_t *>(o + 2 + 4 * sub);    // 2-byte aligned
        o16[0] = (uint16_t)packed;
        o16[1] = (uint16_t)(packed >> 16);
        if (sub == 0) *reinterpret_cast<uint16_t *>(o) = (uint16_t)d16;
    } else {
        reinterpret_cast<uint32_t *>(qs)[t] = packed;  // qs[n][32b + 4sub]
        if (sub == 0) {
            dout[blk] = h2f(d16);
            if (d16out) {                              // block-major fp16 copy [nb][Np] (the LDS GEMM)
                const int64_t nb = K / QK, Np = (N + 3) & ~(int64_t)3;   // 8-byte aligned block rows
                d16out[(blk % nb) * Np + blk / nb] = (uint16_t)d16;
            }
        }
    }
}

hipError_t quantize_q8_0_aos(const float *x, int64_t K, int64_t N, void *xq8, hipStream_t s) {
    const int64_t total8 = N * (K / QK) * 8;
    if (total8 == 0) return hipSuccess;
    const int64_t grid = (total8 + 255) / 256;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_quantize_q8_0<true>, dim3((unsigned)grid), dim3(256), 0, s, x, K, total8,
                       (uint8_t *)xq8, (int8_t *)nullptr, (float *)nullptr, (uint16_t *)nullptr, N);
    return hipGetLastError();
}

hipError_t quantize_q8_0_soa(const float *x, int64_t K, int64_t N, int8_t *qs, float *d, hipStream_t s,
                             uint16_t *d16) {
    const int64_t total8 = N * (K / QK) * 8;
    if (total8 == 0) return hipSuccess;
    const int64_t grid = (total8 + 255) / 256;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_quantize_q8_0<false>, dim3((unsigned)grid), dim3(256), 0, s, x, K, total8,
                       (uint8_t *)nullptr, qs, d, d16, N);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// A3: q4_0 weight quantizer (for synthesising weights on device).  One lane per block.

__global__ __launch_bounds__(256) void k_quantize_q4_0(const float *__restrict__ w, int64_t nblocks,
                                                         uint8_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const float4 *src = reinterpret_cast<const float4 *>(w + i * QK);
    float v[QK];
#pragma unroll
    for (int j = 0; j < QK / 4; j++) {
        const float4 f = src[j];
        v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
    }
    float amax = 0.0f, vmax = 0.0f;
#pragma unroll
    for (int j = 0; j < QK; j++) {
        if (amax < fabsf(v[j])) { amax = fabsf(v[j]); vmax = v[j]; }     // first occurrence wins
    }
    const float d = vmax / -8.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    uint16_t *o16 = reinterpret_cast<uint16_t *>(out + i * Q4B);          // 2-byte aligned
    o16[0] = (uint16_t)f2h(d);
#pragma unroll
    for (int j = 0; j < QK / 2; j += 2) {
        uint32_t b2 = 0;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            // separate rounding of v*id and +8.5 (built with -ffp-contract=off), as the C reference
            int q0 = (int)(signed char)(int)(v[j + t] * id + 8.5f);
            int q1 = (int)(signed char)(int)(v[j + t + QK / 2] * id + 8.5f);
            q0 = q0 > 15 ? 15 : q0;
            q1 = q1 > 15 ? 15 : q1;
            b2 |= (uint32_t)((q0 & 0xFF) | ((q1 & 0xFF) << 4)) << (8 * t);
        }
        o16[1 + j / 2] = (uint16_t)b2;
    }
}

hipError_t quantize_q4_0(const float *w, int64_t K, int64_t M, void *wq, hipStream_t s) {
    const int64_t nblocks = M * (K / QK);
    if (nblocks == 0) return hipSuccess;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_quantize_q4_0, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, s, w, nblocks,
                       (uint8_t *)wq);
    return hipGetLastError();
}

// A4
__global__ __launch_bounds__(256) void k_dequantize_q4_0(const uint8_t *__restrict__ wq, int64_t nblocks,
                                                           float *__restrict__ w) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one lane per (block, byte j)
    if (t >= nblocks * 16) return;
    const int64_t i = t >> 4;
    const int j = (int)(t & 15);
    const uint8_t *b = wq + i * Q4B;
    const float d = h2f((uint32_t)b[0] | ((uint32_t)b[1] << 8));
    const uint8_t q = b[2 + j];
    w[i * QK + j] = (float)((int)(q & 0x0F) - 8) * d;
    w[i * QK + j + 16] = (float)((int)(q >> 4) - 8) * d;
}

hipError_t dequantize_q4_0(const void *wq, int64_t K, int64_t M, float *w, hipStream_t s) {
    const int64_t nblocks = M * (K / QK);
    if (nblocks == 0) return hipSuccess;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_dequantize_q4_0, dim3((unsigned)((nblocks * 16 + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t *)wq, nblocks, w);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// GEMV (decode, N <= 8).
//
// Lane p of a wave owns block pair p of a weight row (and p+64, p+128, ... with row items).  A
// pair is 36 bytes (9 dwords): the 18-byte blocks of a row start 4-byte aligned every second
// block, so a pair is always dword aligned and the 64 lanes of one load read 2,304 contiguous
// bytes (a whole K=4096 row).  Production loads are global_load_dwordx4/x4/x1 with clamped lane
// addresses (VAR bit 0); the descriptor form (out-of-row lanes read 0) is the VAR 0 A/B arm.  The
// even block's qs are re-aligned with v_alignbyte_b32.  x is quantized once per workgroup into
// LDS (q8_0 ints + fp32 d + 8*sum(q)); the q4_0 nibbles enter v_dot4c_i32_i8 unsigned (0..15)
// and the -8 offset is applied once per block as -8*sum(q):  sum((n-8)*q) = sum(n*q) - 8*sum(q).
//
// Schedule: the x-waves load + quantize x while every other wave already streams its first
// DEPTH items; after the barrier each wave walks its items (whole rows with PPL > 0, 64-pair
// chunks otherwise) with DEPTH items in flight.  Launch policy (grid, row mapping, depth, row
// items) in launch_gemv_w / launch_gemv; every policy gives bitwise-identical results.

static constexpr int GEMV_LDS_MAX = 64 * 1024;
// diagnostic build (GGML_HIP_GEMV_DIAG=7): per-wave s_memrealtime stamps of the phases
__device__ unsigned long long g_gemv_stamps[8192 * 8];
#define GEMV_STAMP(slot)                                                                         \
    do {                                                                                         \
        if (DIAG == 7 && lane == 0) {                                                            \
            const int wid_ = blockIdx.x * WAVES + wave;                                          \
            if (wid_ < 8192) g_gemv_stamps[wid_ * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                        \
    } while (0)
static constexpr int GEMV_PRO = 4;          // activation float4 loads in flight per thread
#ifndef GEMV_XPRO_DEF
#define GEMV_XPRO_DEF 4
#endif
static constexpr int GEMV_XPRO = GEMV_XPRO_DEF;   // per x-wave thread in the split prologue
static constexpr int GEMV_MAXMAT = 4;       // sibling matrices per launch

__device__ __forceinline__ int dot_q4_q8(uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3,
                                         const u32x4 xl /* elems 0..15 */, const u32x4 xh /* 16..31 */) {
    const uint32_t m = 0x0F0F0F0Fu;
    int s = 0;
    s = __builtin_amdgcn_sdot4((int)(q0 & m), (int)xl.x, s, false);
    s = __builtin_amdgcn_sdot4((int)(q1 & m), (int)xl.y, s, false);
    s = __builtin_amdgcn_sdot4((int)(q2 & m), (int)xl.z, s, false);
    s = __builtin_amdgcn_sdot4((int)(q3 & m), (int)xl.w, s, false);
    s = __builtin_amdgcn_sdot4((int)((q0 >> 4) & m), (int)xh.x, s, false);
    s = __builtin_amdgcn_sdot4((int)((q1 >> 4) & m), (int)xh.y, s, false);
    s = __builtin_amdgcn_sdot4((int)((q2 >> 4) & m), (int)xh.z, s, false);
    s = __builtin_amdgcn_sdot4((int)((q3 >> 4) & m), (int)xh.w, s, false);
    return s;
}

struct PairRegs {
    u32x4 a, b;
    uint32_t c;
};

__device__ __forceinline__ PairRegs load_pair(const uint8_t *row, int64_t rowbytes, int p) {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(row, (uint32_t)rowbytes);
    PairRegs v;
    v.a = __builtin_amdgcn_raw_buffer_load_b128(r, 36 * p, 0, 0);
    v.b = __builtin_amdgcn_raw_buffer_load_b128(r, 36 * p + 16, 0, 0);
    v.c = __builtin_amdgcn_raw_buffer_load_b32(r, 36 * p + 32, 0, 0);
    return v;
}

// Global-load form: lanes past the row's last pair (and whole past-the-end items) clamp to one
// address, so they add no traffic; no descriptor setup per item.
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
__device__ __forceinline__ PairRegs load_pair_g(const uint8_t *p36) {
    PairRegs v;                                     // global_load (not flat: no lgkmcnt coupling)
    v.a = *(g_u32x4 *)(p36);
    v.b = *(g_u32x4 *)(p36 + 16);
    v.c = *(g_u32 *)(p36 + 32);
    return v;
}

// Up to GEMV_MAXMAT weight matrices that share the activation x ("siblings": wq/wk/wv, w1/w3)
// run as one launch; their rows are concatenated and each (row, chunk) item looks up its matrix.
struct GemvMats {
    const uint8_t *W[GEMV_MAXMAT];
    float *y[GEMV_MAXMAT];
    int64_t ldy[GEMV_MAXMAT];
    int row_begin[GEMV_MAXMAT + 1];       // prefix sums of M; unused entries = total rows
    int n;
    int M;                                // total rows (= row_begin[n])
    int rstride;                          // rows between a wave's consecutive rows = grid * WAVES
    int map;                              // row -> (workgroup, wave) mapping, see the kernel
};
// Every field is read with a constant index: the kernel's kernargs arrive in one batch of scalar
// loads and the per-row matrix lookup is a chain of s_cselect, not a dependent kernarg load.

// Kernel arguments.  Everything a wave needs before its first weight issue (and x for the x-waves)
// comes first as 14 dwords of scalar arguments, which the library build preloads into SGPRs at wave
// start (-mllvm -amdgpu-kernarg-preload-count, Makefile): no kernarg round trip, no branch on a
// kernarg load, no hidden-argument load for the grid size.  Before this the prologue waited on four
// dependent kernarg loads and a 64-bit division (~0.7 us from wave start to the first weight issue in
// the phase stamps).  The rest (a fourth sibling's matrix, y, ldy) is only needed at a row's end.
struct GemvTail {
    const uint8_t *W3;
    float *y[GEMV_MAXMAT];
    int64_t ldy[GEMV_MAXMAT];
    GemvNorm nrm;                         // NORM instantiations only
};
// geom = nb | map << 16 | grid << 18  (nb < 2^16, grid < 2^14; checked by the launcher)

// VAR bit 0 (GLB): weight loads are plain global loads with clamped lane addresses
// VAR bit 1 (XSPLIT): only the first XW waves load and quantize x; the other waves issue their
//                     weight loads at once (the x loads enter the CU's queue first)
// VAR bit 2 (XFIRST, with XSPLIT): a workgroup barrier between the x-waves' x load ISSUE and every
//                     wave's first weight issue, so the x loads are ahead of all of the workgroup's
//                     weight loads in the CU's memory pipeline (phase stamps: without it the x data
//                     returned together with the weights, and the prologue barrier gated compute)
// VAR bit 3 (XHOLD, with XFIRST): the x-waves issue their own weight loads only after x is in LDS
//                     (the other waves stream weights from the start)
// PPL > 0 ("row items", decode, K <= 12288): lane l takes pairs l, l+64, ..., l+64*(PPL-1) of the
//                     row (PPL = ceil(pairs/64)), so one item is a whole row: all of its loads are
//                     in flight together and it is reduced once (a row of K=4160 no longer costs two
//                     items for one extra pair).  PPL == 0: 64-pair chunks, one item per chunk.
// BAL (PPL == 0, NT == 1, PRO == 0; long rows, K > 12288): the row-granular mappings leave a tail
//                     when M is a little above the wave count (Falcon-7B's 18176 -> 4544: 4544 rows on
//                     4096 waves, so 448 waves stream two whole rows while the rest stream one).  BAL
//                     balances at chunk granularity instead: workgroup b owns the blocked row range,
//                     its (row, chunk) items go round-robin to its waves (item i -> wave i % WAVES),
//                     every item is reduced across its lanes on its own and its sum parked in LDS, and
//                     after one workgroup barrier thread t adds row t's chunk sums in chunk order.
//                     Deterministic (no atomics, fixed order), but a different fp32 summation order
//                     from the row-granular policies (within the same oracle bound, not bitwise).
__device__ __forceinline__ double wave_sum_d64(double v) {   // every lane gets the sum
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NT, int DIAG, int WAVES, int DEPTH, int VAR = 0, int PPL = 0, int PRO = 0, int BAL = 0>
__global__ __launch_bounds__(WAVES * 64) void k_gemv_q4_0(const float *__restrict__ x_, const uint8_t *W0,
                                                          const uint8_t *W1, const uint8_t *W2, int rb1_, int rb2_,
                                                          int rb3_, int rowbytes_, int geom, int M_,
                                                          const GemvTail tail) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = geom & 0xFFFF;
    const int map = (geom >> 16) & 3;
    const int grid = (int)((uint32_t)geom >> 18);
    const int64_t rowbytes = rowbytes_;
    // xq: per token, chunk-major [4][npairs] x 16 B: chunk j = (block & 1) * 2 + word / 4 of pair
    // p = block / 2, so lane p's four ds_read_b128 are lane-contiguous (no bank conflicts)
    uint32_t *xq = lds;                                             // [NT][4][npairs][4] int8x4
    float *xd = reinterpret_cast<float *>(lds + NT * nb * 8);      // [NT][nb]
    int *xs = reinterpret_cast<int *>(xd + NT * nb);               // [NT][nb] 8*sum(q)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the y / ldy choice at a row's end is written as sums of deltas selected by (row >=
    // row_begin[i]) so that it compiles to s_cselect (a ternary chain over four struct fields is
    // turned into a lookup table in scratch by the optimizer)
    // (every argument is copied into a local first: a lambda capturing an SGPR-preloaded argument or
    // the by-value struct by reference materialises the whole argument block in scratch)
    const float *const x = x_;
    const uint8_t *const w0 = W0, *const w3 = tail.W3;
    const uint64_t wd1 = (uint64_t)W1 - (uint64_t)W0, wd2 = (uint64_t)W2 - (uint64_t)W1;
    const int rb1 = rb1_, rb2 = rb2_, rb3 = rb3_, M = M_;
    const uint64_t y0 = (uint64_t)tail.y[0], yd1 = (uint64_t)tail.y[1] - (uint64_t)tail.y[0],
                   yd2 = (uint64_t)tail.y[2] - (uint64_t)tail.y[1], yd3 = (uint64_t)tail.y[3] - (uint64_t)tail.y[2];
    const int64_t l0 = tail.ldy[0], ld1 = tail.ldy[1] - tail.ldy[0], ld2 = tail.ldy[2] - tail.ldy[1],
                  ld3 = tail.ldy[3] - tail.ldy[2];
    const int npairs = nb >> 1;
    const int nchunk = PPL > 0 ? 1 : (npairs + 63) >> 6;
    constexpr int NPR = PPL > 0 ? PPL : 1;                          // pairs per lane per item
    struct ItemRegs {
        PairRegs pr[NPR];
    };
    // row -> (workgroup b, wave w) mapping (kernarg `map`):
    //  0 strided:     rows b*WAVES + w + k*grid*WAVES (16 consecutive rows per workgroup pass)
    //  1 interleaved: rows (k*WAVES + w)*grid + b
    //  2 blocked:     workgroup b owns the contiguous range [b*M/grid, (b+1)*M/grid), waves stride 16
    // With grid a multiple of the CU count, 1 and 2 give every CU floor or ceil of M/grid rows per
    // workgroup (no CU streams twice the bytes of another at the tail); 0 does when M is a
    // multiple of grid*WAVES.
    int row0, rstride, rend;
    if (map == 2) {                                                 // grid * M < 2^32 (launcher)
        row0 = (int)(((uint32_t)blockIdx.x * (uint32_t)M) / (uint32_t)grid) + wave;
        rend = (int)(((uint32_t)(blockIdx.x + 1) * (uint32_t)M) / (uint32_t)grid);
        rstride = WAVES;
    } else {
        row0 = map == 1 ? wave * grid + blockIdx.x : blockIdx.x * WAVES + wave;
        rend = M;
        rstride = grid * WAVES;
    }
    static_assert(!BAL || (PPL == 0 && NT == 1 && PRO == 0), "balanced items: decode chunk form only");
    const int rbeg = row0 - wave;                                   // BAL: the workgroup's blocked range
    const int nwg_items = BAL ? (rend - rbeg) * nchunk : 0;         // BAL: (row, chunk) items of the WG
    const int nrows_w = row0 < rend ? (int)((uint32_t)(rend - 1 - row0) / (uint32_t)rstride) + 1 : 0;
    const int nitems = BAL ? (wave < nwg_items ? (nwg_items - 1 - wave) / WAVES + 1 : 0)
                           : nrows_w * nchunk;                      // (row, chunk) items of this wave
    GEMV_STAMP(0);

    static_assert(GEMV_MAXMAT == 4, "matrix selection below is written for 4 siblings");
    auto row_ptr = [&](int r) __attribute__((always_inline)) {     // wave-uniform
        // sums of selected deltas (a ternary chain over the pointers becomes a scratch lookup table)
        const bool g1 = r >= rb1, g2 = r >= rb2;
        uint64_t w = (uint64_t)w0 + (g1 ? wd1 : 0) + (g2 ? wd2 : 0);
        int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0);
        if (r >= rb3) {                       // a fourth sibling: its pointer is not preloaded, and
            asm volatile("");                 // the branch must stay one (a select would wait for it)
            w = (uint64_t)w3;
            rb = rb3;
        }
        return reinterpret_cast<const uint8_t *>(w) + (int64_t)(r - rb) * rowbytes;
    };

    // ---- INIT: q8_0 of the NT activation rows into LDS, first weight chunk issued in between.
    // x of the NT tokens is contiguous ([NT][K] f32), so thread t's float4 is at byte 16*t.  All
    // loads are unconditional buffer loads (out-of-range -> 0, no traffic) so the compiler can
    // count vmcnt exactly: the q8_0 math waits for the activations only, not the weights.
    const int total = NT * nb * 8;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, (uint32_t)total * 16u);
    auto quantize_into_lds = [&](const u32x4 &raw, int t) __attribute__((always_inline)) {
        if (t < total) {                                            // whole 8-lane groups agree
            const float4 v = make_float4(__uint_as_float(raw.x), __uint_as_float(raw.y),
                                         __uint_as_float(raw.z), __uint_as_float(raw.w));
            uint32_t d16;
            int qsum;
            const uint32_t packed = q8_block_lane(v, d16, qsum);
            {
                const int n = t / (nb * 8), tw = t - n * (nb * 8);  // token, word within token
                const int b = tw >> 3, w = tw & 7;
                xq[n * nb * 8 + ((((b & 1) << 1) | (w >> 2)) * (nb >> 1) + (b >> 1)) * 4 + (w & 3)] = packed;
            }
            if ((t & 7) == 0) {
                xd[t >> 3] = h2f(d16);
                xs[t >> 3] = 8 * qsum;
            }
        }
    };
    auto item_row = [&](int it) __attribute__((always_inline)) {
        return BAL ? rbeg + (wave + WAVES * it) / nchunk : row0 + (it / nchunk) * rstride;
    };
    auto item_chunk = [&](int it) __attribute__((always_inline)) {
        return BAL ? (wave + WAVES * it) % nchunk : it % nchunk;
    };
    constexpr bool GLB = (VAR & 1) != 0, XSPLIT = (VAR & 2) != 0, XFIRST = (VAR & 4) != 0, XHOLD = (VAR & 8) != 0;
    static_assert(PPL == 0 || GLB, "row items use the global-load form");
    auto issue = [&](int it) __attribute__((always_inline)) {
        const bool valid = it < nitems;                             // past the end: zero-size descriptor
        const int r = valid ? item_row(it) : row0;
        ItemRegs v;
        if constexpr (GLB) {                                        // past the end: one shared address
            const uint8_t *rp = row_ptr(valid ? r : 0);
#pragma unroll
            for (int j = 0; j < NPR; j++) {
                const int pp = 64 * (PPL > 0 ? j : item_chunk(it)) + lane;
                const int pc = valid ? (pp < npairs ? pp : npairs - 1) : 0;
                v.pr[j] = load_pair_g(rp + 36 * pc);
            }
        } else {
            v.pr[0] = load_pair(row_ptr(valid ? r : 0), valid ? rowbytes : 0, 64 * item_chunk(it) + lane);
        }
        return v;
    };
    constexpr bool KO_X = DIAG == 8 || DIAG == 10;      // timing knockouts (results invalid)
    constexpr bool KO_LDS = DIAG == 9 || DIAG == 10;
    u32x4 xv[GEMV_PRO];
    ItemRegs buf[DEPTH];
    if constexpr (PRO == 2) {
        // silu -> mul fused into the x prologue (NT == 1, one round of x-waves; see GemvNorm)
        static_assert(NT == 1 && XSPLIT, "silu prologue: decode x-wave form only");
        const int XW = (total + 64 * GEMV_XPRO - 1) / (64 * GEMV_XPRO);
        const int XT = XW * 64;
        const GemvNorm nrm = tail.nrm;
        if (wave < XW) {
            const __amdgpu_buffer_rsrc_t ar = make_rsrc(nrm.a, (uint32_t)total * 16u);
            u32x4 rb[GEMV_XPRO], ra[GEMV_XPRO];
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                rb[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (tid + i * XT), 0, 0);
                ra[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, 16 * (tid + i * XT), 0, 0);
            }
            if constexpr (!XHOLD) {
#pragma unroll
                for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
            }
            typedef __attribute__((address_space(1))) const uint16_t g_u16;
            const bool store = blockIdx.x == 0;
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                const int idx = tid + i * XT;
                if (idx < total) {
                    const uint32_t av[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
                    const uint32_t bv[4] = {rb[i].x, rb[i].y, rb[i].z, rb[i].w};
                    float u[4], o[4];
#pragma unroll
                    for (int c = 0; c < 4; c++) {    // as k_silu_mul: s = table[fp16(a)], out = s * b
                        u[c] = h2f(((g_u16 *)nrm.table)[f2h(__uint_as_float(av[c]))]);
                        o[c] = u[c] * __uint_as_float(bv[c]);
                    }
                    if (store) {
                        if (nrm.norm) reinterpret_cast<float4 *>(nrm.norm)[idx] = make_float4(u[0], u[1], u[2], u[3]);
                        if (nrm.out) reinterpret_cast<float4 *>(nrm.out)[idx] = make_float4(o[0], o[1], o[2], o[3]);
                    }
                    quantize_into_lds(u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]),
                                            __float_as_uint(o[3])}, idx);
                }
            }
            if constexpr (XHOLD) {
#pragma unroll
                for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
            }
        } else {
#pragma unroll
            for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
        }
        GEMV_STAMP(1);
        GEMV_STAMP(2);
    } else if constexpr (PRO == 1) {
        // [add ->] rms_norm -> mul fused into the x prologue (NT == 1, one round of x-waves: the
        // launcher checks K <= 16 * 64 * 4 * GEMV_XPRO).  The x-waves hold the row in registers, sum
        // its squares in double (order-free in practice, as k_row_norm4's), exchange the per-wave
        // sums through LDS (one extra workgroup barrier), then scale, multiply by the norm weight and
        // quantize; workgroup 0 also stores the chain's tensors.
        static_assert(NT == 1 && XSPLIT, "norm prologue: decode x-wave form only");
        double *npart = reinterpret_cast<double *>(xs + NT * nb);
        const int XW = (total + 64 * GEMV_XPRO - 1) / (64 * GEMV_XPRO);
        const int XT = XW * 64;
        const GemvNorm nrm = tail.nrm;
        float4 v[GEMV_XPRO];
        u32x4 rg[GEMV_XPRO];                                   // the norm weight, loaded with x
        if (wave < XW) {
            const __amdgpu_buffer_rsrc_t ar = make_rsrc(nrm.a ? (const void *)nrm.a : (const void *)x,
                                                        nrm.a ? (uint32_t)total * 16u : 0u);
            const __amdgpu_buffer_rsrc_t gr = make_rsrc(nrm.w, (uint32_t)total * 16u);
            u32x4 rb[GEMV_XPRO], ra[GEMV_XPRO];
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                rb[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (tid + i * XT), 0, 0);
                ra[i] = __builtin_amdgcn_raw_buffer_load_b128(ar, 16 * (tid + i * XT), 0, 0);
                rg[i] = __builtin_amdgcn_raw_buffer_load_b128(gr, 16 * (tid + i * XT), 0, 0);
            }
            if constexpr (!XHOLD) {
#pragma unroll
                for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
            }
            double ss = 0.0;
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                float4 b4 = make_float4(__uint_as_float(rb[i].x), __uint_as_float(rb[i].y), __uint_as_float(rb[i].z),
                                        __uint_as_float(rb[i].w));
                if (nrm.a)                                     // a + b, as k_add_f32 / k_row_norm4
                    b4 = make_float4(__uint_as_float(ra[i].x) + b4.x, __uint_as_float(ra[i].y) + b4.y,
                                     __uint_as_float(ra[i].z) + b4.z, __uint_as_float(ra[i].w) + b4.w);
                v[i] = b4;                                     // past the row: 0 (descriptor)
                ss += (double)(b4.x * b4.x);
                ss += (double)(b4.y * b4.y);
                ss += (double)(b4.z * b4.z);
                ss += (double)(b4.w * b4.w);
            }
            ss = wave_sum_d64(ss);
            if (lane == 0) npart[wave] = ss;
        } else {
#pragma unroll
            for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
        }
        GEMV_STAMP(1);
        __syncthreads();                                       // the per-wave sums
        if (wave < XW) {
            double t = 0.0;
            for (int i = 0; i < XW; i++) t += npart[i];
            const float mean = (float)(t / (double)(nb * QK));
            const float scale = 1.0f / (float)__builtin_sqrt((double)(mean + 1e-6f));
            const bool store = blockIdx.x == 0;
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                const int idx = tid + i * XT;
                if (idx < total) {
                    const float4 xv4 = v[i];
                    const float4 y = make_float4(xv4.x * scale, xv4.y * scale, xv4.z * scale, xv4.w * scale);
                    const float4 g = make_float4(__uint_as_float(rg[i].x), __uint_as_float(rg[i].y),
                                                 __uint_as_float(rg[i].z), __uint_as_float(rg[i].w));
                    const float4 o = make_float4(y.x * g.x, y.y * g.y, y.z * g.z, y.w * g.w);
                    if (store) {
                        if (nrm.sum) reinterpret_cast<float4 *>(nrm.sum)[idx] = xv4;
                        if (nrm.norm) reinterpret_cast<float4 *>(nrm.norm)[idx] = y;
                        if (nrm.out) reinterpret_cast<float4 *>(nrm.out)[idx] = o;
                    }
                    quantize_into_lds(u32x4{__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z),
                                            __float_as_uint(o.w)}, idx);
                }
            }
            if constexpr (XHOLD) {
#pragma unroll
                for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
            }
        }
        GEMV_STAMP(2);
    } else if constexpr (XSPLIT) {
        // x-waves: wave < XW load + quantize x (XT threads, PRO float4 each per round), then issue
        // their weight loads; the other waves only issue weight loads
        const int XW0 = (total + 64 * GEMV_XPRO - 1) / (64 * GEMV_XPRO);
        const int XW = XW0 < WAVES ? XW0 : WAVES;
        const int XT = XW * 64;
        if constexpr (XFIRST) {
            u32x4 xw[GEMV_XPRO];
            if (wave < XW) {
#pragma unroll
                for (int i = 0; i < GEMV_XPRO; i++)
                    xw[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (tid + i * XT), 0, 0);
            }
            __builtin_amdgcn_s_barrier();                           // x loads issued before any weight
            asm volatile("" ::: "memory");
            if (!XHOLD || wave >= XW) {
#pragma unroll
                for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
            }
            GEMV_STAMP(1);
            if (wave < XW) {
#pragma unroll
                for (int i = 0; i < GEMV_XPRO; i++) quantize_into_lds(xw[i], tid + i * XT);
                for (int base = GEMV_XPRO * XT; base < total; base += GEMV_XPRO * XT) {
#pragma unroll
                    for (int i = 0; i < GEMV_XPRO; i++)
                        xw[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * XT), 0, 0);
#pragma unroll
                    for (int i = 0; i < GEMV_XPRO; i++) quantize_into_lds(xw[i], base + tid + i * XT);
                }
                // XHOLD: an x-wave's own weight loads enter the CU's queue only after x is in LDS.
                // Issue blocks once ~30-40 KB per CU are outstanding (phase stamps), so a wave that
                // issued its weights first would sit behind them before it could quantize.
                if constexpr (XHOLD) {
#pragma unroll
                    for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
                }
            }
        } else if (wave < XW) {
            u32x4 xw[GEMV_XPRO];
            for (int base = 0; base < total; base += GEMV_XPRO * XT) {
#pragma unroll
                for (int i = 0; i < GEMV_XPRO; i++)
                    xw[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * XT), 0, 0);
#pragma unroll
                for (int i = 0; i < GEMV_XPRO; i++) quantize_into_lds(xw[i], base + tid + i * XT);
            }
            asm volatile("" ::: "memory");                          // weight loads stay behind x
#pragma unroll
            for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
        } else {
#ifdef GEMV_WSLEEP
            __builtin_amdgcn_s_sleep(GEMV_WSLEEP);                   // A/B knob: x loads enter first
#endif
#pragma unroll
            for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
        }
        if constexpr (!XFIRST) GEMV_STAMP(1);
        GEMV_STAMP(2);
    } else {
#pragma unroll
    for (int i = 0; i < GEMV_PRO; i++)
        xv[i] = KO_X ? u32x4{0, 0, 0, 0} : __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (tid + i * (WAVES * 64)), 0, 0);
    // the wave's first DEPTH items are in flight across the prologue (a ring of named register
    // sets, never copied: a copy would force a wait on the loads still in flight)
#pragma unroll
    for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
    GEMV_STAMP(1);
    if (!KO_X) {
#pragma unroll
    for (int i = 0; i < GEMV_PRO; i++) quantize_into_lds(xv[i], tid + i * (WAVES * 64));
    }
    GEMV_STAMP(2);
    for (int base = GEMV_PRO * (WAVES * 64); !KO_X && base < total; base += GEMV_PRO * (WAVES * 64)) {
#pragma unroll
        for (int i = 0; i < GEMV_PRO; i++)
            xv[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * (WAVES * 64)), 0, 0);
#pragma unroll
        for (int i = 0; i < GEMV_PRO; i++) quantize_into_lds(xv[i], base + tid + i * (WAVES * 64));
    }
    }
    if (!KO_X) __syncthreads();
    GEMV_STAMP(3);

    // ---- COMPUTE: stream the wave's items with DEPTH items in flight in a ring of named register
    // sets (no register copies: a copy would force a wait on the in-flight loads).
    float acc[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) acc[n] = 0.0f;
    float *const part = reinterpret_cast<float *>(xs + NT * nb);   // BAL: [rows of the WG][nchunk]
    auto process = [&](const ItemRegs &vi, int it) __attribute__((always_inline)) {
        const int chunk = item_chunk(it);
#pragma unroll
        for (int j = 0; j < NPR; j++) {
        const PairRegs &v = vi.pr[j];
        const int p = 64 * (PPL > 0 ? j : chunk) + lane;
        if (p < npairs) {
            // even block 2p: d = a.x[15:0], qs = bytes 2..17 ; odd block 2p+1: d = b.x[31:16], qs = b.y..c
            const float dA = h2f(v.a.x & 0xFFFFu);
            const float dB = h2f(v.b.x >> 16);
            const uint32_t qA0 = __builtin_amdgcn_alignbyte(v.a.y, v.a.x, 2);
            const uint32_t qA1 = __builtin_amdgcn_alignbyte(v.a.z, v.a.y, 2);
            const uint32_t qA2 = __builtin_amdgcn_alignbyte(v.a.w, v.a.z, 2);
            const uint32_t qA3 = __builtin_amdgcn_alignbyte(v.b.x, v.a.w, 2);
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const int bA = n * nb + 2 * p;
                const float2 dx = KO_LDS ? make_float2(1.0f, 2.0f) : *reinterpret_cast<const float2 *>(xd + bA);
                const int2 sx = KO_LDS ? make_int2(0, 0) : *reinterpret_cast<const int2 *>(xs + bA);
                const u32x4 *xc = reinterpret_cast<const u32x4 *>(xq + n * nb * 8) + p;
                const u32x4 c1{0x01010101u, 0x02020202u, 0x03030303u, (uint32_t)p};
                const int sA = dot_q4_q8(qA0, qA1, qA2, qA3, KO_LDS ? c1 : xc[0], KO_LDS ? c1 : xc[npairs]) - (KO_LDS ? p : sx.x);
                const int sB = dot_q4_q8(v.b.y, v.b.z, v.b.w, v.c, KO_LDS ? c1 : xc[2 * npairs], KO_LDS ? c1 : xc[3 * npairs]) - (KO_LDS ? lane : sx.y);
                acc[n] = fmaf((float)sA, dA * dx.x, acc[n]);
                acc[n] = fmaf((float)sB, dB * dx.y, acc[n]);
            }
        }
        }
        if constexpr (BAL) {                                        // this item's sum -> LDS
            const float t = wave_sum_lane63(acc[0]);
            if (lane == 63) part[wave + WAVES * it] = t;
            acc[0] = 0.0f;
        } else if (chunk == nchunk - 1) {                           // row complete: reduce + store
            const int r = item_row(it);
            const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
            const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
            // global (not flat) store: a flat store also counts in lgkmcnt, so the next item's LDS
            // waits would wait for its memory round trip
            typedef __attribute__((address_space(1))) float gfloat;
            gfloat *yo = reinterpret_cast<gfloat *>(y0 + (g1 ? yd1 : 0) + (g2 ? yd2 : 0) + (g3 ? yd3 : 0)) + (r - rb);
            const int64_t ld = l0 + (g1 ? ld1 : 0) + (g2 ? ld2 : 0) + (g3 ? ld3 : 0);
            float out = 0.0f;
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const float t = wave_sum_lane63(acc[n]);
                const float tn = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 63));
                out = (lane == n) ? tn : out;
                acc[n] = 0.0f;
            }
            if (lane < NT) yo[(int64_t)lane * ld] = out;
        }
    };
    for (int it = 0; it < nitems; it += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            if (it + d >= nitems) break;
            if (DIAG == 7 && it + d == 0) {                         // when the first weights have landed
                asm volatile("" ::"v"(buf[0].pr[0].a), "v"(buf[0].pr[0].b), "v"(buf[0].pr[0].c));
                GEMV_STAMP(4);
            }
            process(buf[d], it + d);
            if (it + d == 0) GEMV_STAMP(5);
            buf[d] = issue(it + d + DEPTH);
        }
    }
    if constexpr (BAL) {                                            // rows' chunk sums, in chunk order
        __syncthreads();
        typedef __attribute__((address_space(1))) float gfloat;
        for (int rr = tid; rr < rend - rbeg; rr += WAVES * 64) {
            float out = 0.0f;
            for (int c = 0; c < nchunk; c++) out += part[rr * nchunk + c];
            const int r = rbeg + rr;
            const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
            const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
            gfloat *yo = reinterpret_cast<gfloat *>(y0 + (g1 ? yd1 : 0) + (g2 ? yd2 : 0) + (g3 ? yd3 : 0)) + (r - rb);
            *yo = out;
        }
    }
    GEMV_STAMP(6);
}

static int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

// GEMV launch policy overrides: -1 / 0 = automatic.  Initialised from the environment
// (GGML_HIP_GEMV_MAP / _DEPTH / _ROWITEMS / _WG_PER_CU) and settable at run time by the
// non-header debug entry point ggml_hip_debug_set_gemv_policy (tests sweep every path).
struct GemvPolicy {
    int map, depth, rowitems, wg_per_cu, bal;
};
static GemvPolicy &gemv_policy() {
    static GemvPolicy p = {env_int("GGML_HIP_GEMV_MAP", -1), env_int("GGML_HIP_GEMV_DEPTH", 0),
                           env_int("GGML_HIP_GEMV_ROWITEMS", 1), env_int("GGML_HIP_GEMV_WG_PER_CU", 0),
                           env_int("GGML_HIP_GEMV_BAL", -1)};
    return p;
}
void gemv_set_policy(int map, int depth, int rowitems, int wg_per_cu) {
    const int bal = gemv_policy().bal;
    gemv_policy() = {map, depth, rowitems, wg_per_cu, bal};
}
void gemv_set_bal(int bal) { gemv_policy().bal = bal; }

int gemv_max_tokens(int64_t K) {
    const int64_t nb = K / QK;
    int nt = 8;
    while (nt > 0 && nt * nb * 40 > GEMV_LDS_MAX) nt--;
    return nt;
}


template <int NT, int DIAG, int WAVES, int DEPTH, int VAR = 0, int PPL = 0, int PRO = 0, int BAL = 0>
static hipError_t launch_gemv_w(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s,
                                const GemvNorm *nrm = nullptr) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    size_t lds = (size_t)NT * nb * 40 + (PRO == 1 ? WAVES * sizeof(double) : 0);
    const int wg_per_cu_env = gemv_policy().wg_per_cu;
    const int64_t M = m.row_begin[m.n];
    const int64_t need = (M + WAVES - 1) / WAVES;
    const int64_t cus = dev.num_cus;
    // one workgroup per CU while that leaves at most two rows per wave (M <= 2*CUs*WAVES: 8192 on
    // MI355X), two (full occupancy) above; measured per shape with tools/shape_sweep.py
    static int occ = 0;                    // resident workgroups per CU for this instantiation
    if (occ == 0) {
        int nb_occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_occ, k_gemv_q4_0<NT, DIAG, WAVES, DEPTH, VAR, PPL, PRO, BAL>,
                                                         WAVES * 64, lds) != hipSuccess || nb_occ < 1)
            nb_occ = 1;
        occ = nb_occ;
    }
    int wg_per_cu = wg_per_cu_env > 0 ? wg_per_cu_env : (M <= 2 * cus * WAVES ? 1 : 2048 / (WAVES * 64));
    if (wg_per_cu > occ) wg_per_cu = occ;  // never more than can be resident (no second round)
    const int64_t cap = cus * (wg_per_cu < 1 ? 1 : wg_per_cu);
    // a multiple of the CU count (balanced per CU) once there is more than one WG's rows per CU
    const int64_t bal = need <= cus ? need : cus * ((need + cus - 1) / cus);
    const unsigned grid = (unsigned)(bal < cap ? bal : cap);
    const int map_env = gemv_policy().map;
    // strided (contiguous 16-row spans) when its leftover rows form whole rounds of one workgroup per
    // CU (every CU then gets the same rows); otherwise interleaved at two workgroups per CU and
    // blocked at one (measured per shape, tools/shape_sweep.py)
    int map = map_env >= 0 ? map_env
            : ((M % ((int64_t)grid * WAVES)) % (cus * WAVES) == 0 ? 0 : ((int64_t)grid > cus ? 1 : 2));
    if (map == 2 && (int64_t)grid * M >= (int64_t)1 << 32) map = 1;   // the kernel's 32-bit row split
    if (BAL) {                           // blocked rows; chunk sums of the workgroup's rows in LDS
        if ((int64_t)grid * M >= (int64_t)1 << 32) return hipErrorInvalidValue;
        map = 2;
        const int64_t nchunk = (nb / 2 + 63) / 64;
        lds += (size_t)((M + grid - 1) / grid) * nchunk * sizeof(float);
        if (lds > GEMV_LDS_MAX) return hipErrorInvalidValue;   // launch_gemv checks before choosing BAL
    }
    if (nb >= (1 << 16) || grid >= (1u << 14) || rowbytes > INT_MAX || M > INT_MAX) return hipErrorInvalidValue;
    GemvTail tail{};
    if (nrm) tail.nrm = *nrm;
    tail.W3 = m.W[3];
    for (int i = 0; i < GEMV_MAXMAT; i++) {
        tail.y[i] = m.y[i];
        tail.ldy[i] = m.ldy[i];
    }
    const int geom = nb | map << 16 | (int)(grid << 18);
    (void)hipGetLastError();  // report only this launch's error
    launch_k((k_gemv_q4_0<NT, DIAG, WAVES, DEPTH, VAR, PPL, PRO, BAL>), dim3(grid), dim3(WAVES * 64), lds, s, x, m.W[0],
                       m.W[1], m.W[2], m.row_begin[1], m.row_begin[2], m.row_begin[3], (int)rowbytes, geom, (int)M, tail);
    return hipGetLastError();
}

#ifndef GEMV_RW
#define GEMV_RW 16
#endif
template <int NT, int DIAG, int VAR>
static hipError_t launch_gemv_rows(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s,
                                   int ppl, int rd) {
    switch (ppl) {
        case 1: return rd == 1 ? launch_gemv_w<NT, DIAG, GEMV_RW, 1, VAR, 1>(m, K, x, dev, s)
                               : launch_gemv_w<NT, DIAG, GEMV_RW, 2, VAR, 1>(m, K, x, dev, s);
        case 2: return rd == 1 ? launch_gemv_w<NT, DIAG, GEMV_RW, 1, VAR, 2>(m, K, x, dev, s)
                               : launch_gemv_w<NT, DIAG, GEMV_RW, 2, VAR, 2>(m, K, x, dev, s);
        default: return rd == 1 ? launch_gemv_w<NT, DIAG, GEMV_RW, 1, VAR, 3>(m, K, x, dev, s)
                                : launch_gemv_w<NT, DIAG, GEMV_RW, 2, VAR, 3>(m, K, x, dev, s);
    }
}

template <int NT>
static hipError_t launch_gemv(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s) {
    // Production: VAR 3 or 15 (global weight loads + x-wave prologue; policy below), decode row items
    // at ring depth 1; chunked items (N > 1 or K > 12288) at depth 1 for single-chunk rows and 2
    // otherwise (measured per shape, tools/gemv_ab.sh).  GGML_HIP_GEMV_VAR=0 / 3 / 7 / 15 and
    // GGML_HIP_GEMV_DEPTH=1|2 select the A/B variants;
    // GGML_HIP_GEMV_DIAG=7 the phase-stamp build (row items as in production), 8/9/10 the timing
    // knockouts (invalid results).
    static const int diag = env_int("GGML_HIP_GEMV_DIAG", 0);
    static const int var_env = env_int("GGML_HIP_GEMV_VAR", -1);
    const int depth_env = gemv_policy().depth;
    // Decode row items (round 2, with preloaded kernargs; tools/gemv_ab.sh, LLaMA-7B shapes): one row
    // in flight per wave, and XHOLD (VAR 15: the x-waves issue their own weights once x is in LDS)
    // when a wave has at most two rows and x is short (wq|wk|wv 7.33 -> 7.19 us, wo 4.82 -> 4.24);
    // VAR 3 otherwise (w1|w3 at 2.7 rows per wave 10.56 vs 10.73, w2 at K = 11008 7.33 vs 8.06)
    const int64_t Mrows = m.row_begin[m.n];
    const int var = var_env >= 0 ? var_env : (NT == 1 && K <= 8192 && Mrows <= 2 * 16 * (int64_t)dev.num_cus * 2 ? 15 : 3);
    const int depth = depth_env ? depth_env : (K / 64 > 64 ? 2 : 1);
    if constexpr (NT == 1) {
        if (diag == 8) return launch_gemv_w<NT, 8, 16, 1>(m, K, x, dev, s);
        if (diag == 9) return launch_gemv_w<NT, 9, 16, 1>(m, K, x, dev, s);
        if (diag == 10) return launch_gemv_w<NT, 10, 16, 1>(m, K, x, dev, s);
    }
    if constexpr (NT == 1) {                        // decode: one item per row (PPL pairs per lane)
        const int rowitems = gemv_policy().rowitems;
        const int ppl = (int)((K / 64 + 63) / 64);
        if (rowitems && (var == 3 || var == 7 || var == 15) && ppl <= 3) {
            // two rows in flight per wave, except the multi-round strided case (M > 2*CUs*16 with
            // the leftover rows a whole round per CU, e.g. the fused LLaMA-7B wq|wk|wv, M = 12288)
            const int rd = depth_env ? depth_env : 1;
            if (diag == 7) return var == 15 ? launch_gemv_rows<NT, 7, 15>(m, K, x, dev, s, ppl, rd)
                                  : var == 7 ? launch_gemv_rows<NT, 7, 7>(m, K, x, dev, s, ppl, rd)
                                             : launch_gemv_rows<NT, 7, 3>(m, K, x, dev, s, ppl, rd);
            return var == 15 ? launch_gemv_rows<NT, 0, 15>(m, K, x, dev, s, ppl, rd)
                 : var == 7 ? launch_gemv_rows<NT, 0, 7>(m, K, x, dev, s, ppl, rd)
                            : launch_gemv_rows<NT, 0, 3>(m, K, x, dev, s, ppl, rd);
        }
        // K > 12288: chunked items below (measured equal or faster at 4-5 pairs per lane), balanced at
        // chunk granularity (BAL) when whole rows per wave leave a long tail: the busiest wave of the
        // row-granular mapping streams ceil(M / waves) rows, a BAL wave ceil(rows per WG * chunks / 16)
        // chunks; BAL when that is at most 0.65 of the rows' chunks (GGML_HIP_GEMV_BAL=0/1 overrides).
        // Measured (tools/r2_bal.sh, 2 rounds): Falcon 18176 -> 4544 14.6 -> 13.2-14.1 us (the bench's
        // Falcon-7B line 845 -> 875 tok/s), LLaMA-13B 13824 -> 5120 11.25 either way, NeoX 24576 -> 6144
        // 20.2 -> 20.9-21.1 (0.75: not taken)
        const int bal_env = gemv_policy().bal;
        if (diag == 0 && var == 3 && bal_env != 0 && ppl > 3) {
            const int64_t cus = dev.num_cus;
            const int64_t wg = gemv_policy().wg_per_cu > 0 ? gemv_policy().wg_per_cu : (Mrows <= 2 * cus * 16 ? 1 : 2);
            const int64_t need = (Mrows + 15) / 16, cap = cus * wg;        // launch_gemv_w's grid rule
            const int64_t bgrid = need <= cus ? need : cus * ((need + cus - 1) / cus);
            const int64_t grid = bgrid < cap ? bgrid : cap, nchunk = (K / 64 + 63) / 64;
            const int64_t rows_w = (Mrows + grid * 16 - 1) / (grid * 16);
            const int64_t items_w = (((Mrows + grid - 1) / grid) * nchunk + 15) / 16;
            const int64_t lds_bal = (K / QK) * 40 + ((Mrows + grid - 1) / grid) * nchunk * 4;
            if (lds_bal <= GEMV_LDS_MAX && (bal_env == 1 || 20 * items_w <= 13 * rows_w * nchunk))
                return depth == 1 ? launch_gemv_w<NT, 0, 16, 1, 3, 0, 0, 1>(m, K, x, dev, s)
                                  : launch_gemv_w<NT, 0, 16, 2, 3, 0, 0, 1>(m, K, x, dev, s);
        }
        if (diag == 7) return depth == 1 ? launch_gemv_w<NT, 7, 16, 1, 3>(m, K, x, dev, s)
                                         : launch_gemv_w<NT, 7, 16, 2, 3>(m, K, x, dev, s);
    }
    if (var == 0) return depth == 1 ? launch_gemv_w<NT, 0, 16, 1, 0>(m, K, x, dev, s)
                                    : launch_gemv_w<NT, 0, 16, 2, 0>(m, K, x, dev, s);
    if (var == 7) return depth == 1 ? launch_gemv_w<NT, 0, 16, 1, 7>(m, K, x, dev, s)
                                    : launch_gemv_w<NT, 0, 16, 2, 7>(m, K, x, dev, s);
    return depth == 1 ? launch_gemv_w<NT, 0, 16, 1, 3>(m, K, x, dev, s)
                      : launch_gemv_w<NT, 0, 16, 2, 3>(m, K, x, dev, s);
}

hipError_t gemv_read_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemv_stamps), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost);
}

hipError_t gemv_q4_0_multi(int nmat, const void *const *W, const int64_t *M, int64_t K, const float *x, int64_t N,
                           float *const *y, const int64_t *ldy, const DeviceInfo &dev, hipStream_t s) {
    if (nmat < 1 || nmat > GEMV_MAXMAT) return hipErrorInvalidValue;
    GemvMats m{};
    m.n = nmat;
    m.row_begin[0] = 0;
    for (int i = 0; i < nmat; i++) {
        m.W[i] = (const uint8_t *)W[i];
        m.y[i] = y[i];
        m.ldy[i] = ldy[i];
        m.row_begin[i + 1] = m.row_begin[i] + (int)M[i];
    }
    for (int i = nmat; i < GEMV_MAXMAT; i++) {
        m.W[i] = m.W[0];
        m.y[i] = m.y[0];
        m.ldy[i] = m.ldy[0];
        m.row_begin[i + 1] = m.row_begin[i];
    }
    switch (N) {
        case 1: return launch_gemv<1>(m, K, x, dev, s);
        case 2: return launch_gemv<2>(m, K, x, dev, s);
        case 3: return launch_gemv<3>(m, K, x, dev, s);
        case 4: return launch_gemv<4>(m, K, x, dev, s);
        case 5: return launch_gemv<5>(m, K, x, dev, s);
        case 6: return launch_gemv<6>(m, K, x, dev, s);
        case 7: return launch_gemv<7>(m, K, x, dev, s);
        case 8: return launch_gemv<8>(m, K, x, dev, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t gemv_q4_0(const void *W, int64_t K, int64_t M, const float *x, int64_t N, float *y, int64_t ldy,
                     const DeviceInfo &dev, hipStream_t s) {
    return gemv_q4_0_multi(1, &W, &M, K, x, N, &y, &ldy, dev, s);
}

template <int VAR, int PPL>
static hipError_t launch_gemv_norm(const GemvMats &m, int64_t K, const float *b, const DeviceInfo &dev, hipStream_t s,
                                   const GemvNorm &nrm, int rd) {
    if (nrm.kind == 2)
        return rd == 2 ? launch_gemv_w<1, 0, 16, 2, VAR, PPL, 2>(m, K, b, dev, s, &nrm)
                       : launch_gemv_w<1, 0, 16, 1, VAR, PPL, 2>(m, K, b, dev, s, &nrm);
    return rd == 2 ? launch_gemv_w<1, 0, 16, 2, VAR, PPL, 1>(m, K, b, dev, s, &nrm)
                   : launch_gemv_w<1, 0, 16, 1, VAR, PPL, 1>(m, K, b, dev, s, &nrm);
}

hipError_t gemv_q4_0_multi_norm(int nmat, const void *const *W, const int64_t *M, int64_t K, const float *b,
                                const GemvNorm &nrm, float *const *y, const int64_t *ldy, const DeviceInfo &dev,
                                hipStream_t s) {
    // one round of x-waves holds the row: K / 4 float4 <= 16 waves * 64 lanes * GEMV_XPRO
    if (nmat < 1 || nmat > GEMV_MAXMAT || K % 64 != 0 || K / 4 > 16 * 64 * GEMV_XPRO || !b ||
        (nrm.kind == 1 && !nrm.w) || (nrm.kind == 2 && (!nrm.a || !nrm.table)) || (nrm.kind != 1 && nrm.kind != 2))
        return hipErrorInvalidValue;
    GemvMats m{};
    m.n = nmat;
    m.row_begin[0] = 0;
    for (int i = 0; i < nmat; i++) {
        m.W[i] = (const uint8_t *)W[i];
        m.y[i] = y[i];
        m.ldy[i] = ldy[i];
        m.row_begin[i + 1] = m.row_begin[i] + (int)M[i];
    }
    for (int i = nmat; i < GEMV_MAXMAT; i++) {
        m.W[i] = m.W[0];
        m.y[i] = m.y[0];
        m.ldy[i] = m.ldy[0];
        m.row_begin[i + 1] = m.row_begin[i];
    }
    // the same policy as launch_gemv<1> (row items, ring depth, VAR 15 for short rows)
    static const int var_env = env_int("GGML_HIP_GEMV_VAR", -1);
    const int depth_env = gemv_policy().depth;
    const int64_t Mrows = m.row_begin[m.n];
    const int var = var_env == 15 || var_env == 3 ? var_env : (K <= 8192 && Mrows <= 2 * 16 * (int64_t)dev.num_cus * 2 ? 15 : 3);
    const int rd = depth_env == 2 ? 2 : 1;
    const int ppl = (int)((K / 64 + 63) / 64);
    if (var == 15) {
        if (ppl == 1) return launch_gemv_norm<15, 1>(m, K, b, dev, s, nrm, rd);
        if (ppl == 2) return launch_gemv_norm<15, 2>(m, K, b, dev, s, nrm, rd);
        if (ppl == 3) return launch_gemv_norm<15, 3>(m, K, b, dev, s, nrm, rd);
    } else {
        if (ppl == 1) return launch_gemv_norm<3, 1>(m, K, b, dev, s, nrm, rd);
        if (ppl == 2) return launch_gemv_norm<3, 2>(m, K, b, dev, s, nrm, rd);
        if (ppl == 3) return launch_gemv_norm<3, 3>(m, K, b, dev, s, nrm, rd);
    }
    return hipErrorInvalidValue;        // K > 12288: chunked items are not instantiated with the prologue
}

// ---------------------------------------------------------------------------------------------
// GEMM (prefill): int8 MFMA v_mfma_i32_32x32x32_i8, K = 32 = one q4_0/q8_0 block per MFMA.
//
// Workgroup = 8 waves, tile 64 weight rows x 128 tokens; wave (wr, wt) in 2 x 4 owns one 32x32
// MFMA tile.  K advances GM_KB = 4 blocks (128 values) per stage through a double-buffered LDS
// ring with one barrier per stage.  Global loads run TWO stages ahead in two named register
// sets (HBM latency under load is ~2 us, longer than one stage of MFMAs); two workgroups per
// CU (16 waves) cover the rest.
//
// Staging converts every weight element once per workgroup: thread t < 128 owns (row t/2,
// block pair t%2) of the stage, loads the pair's 36 raw bytes (dword aligned, as in the GEMV),
// turns the nibbles into int8 (n-8) and writes [block][row][32 B] + fp32 d_w.  Activations arrive
// already q8_0-quantized (int8 qs [N][K] + fp32 d_x, from k_quantize_q8_0<false>).  LDS rows are
// 32 B; the two 16-byte halves of row r are swapped when (r>>3)&1 so that the ds_read_b128 of 32
// consecutive rows hits 16 distinct bank slots per lane group.
//
// MFMA roles: A = activations (token = MFMA row), B = weights (weight row = MFMA column): lane
// (c, h) = (lane&31, lane>>5) supplies k-half h (elements 16h..16h+15) of token c (A) and of
// weight row c (B).  D[token][row] has the weight row on the lane, so each output register is
// a 128-byte contiguous store and d_w is one value per lane.  The i32 MFMA result is the exact
// block sum; the epilogue applies d_x[token] * d_w[row] in fp32 (fmaf per block).

static constexpr int GM_BM = 64, GM_BN = 128, GM_KB = 4, GM_WAVES = 8, GM_THREADS = GM_WAVES * 64;
static constexpr int GM_STAGE_W = GM_KB * GM_BM * 32;          // int8 weights  [KB][BM][32]
static constexpr int GM_STAGE_X = GM_KB * GM_BN * 32;          // int8 acts     [KB][BN][32]
static constexpr int GM_STAGE_WD = GM_KB * GM_BM * 4;          // f32 d_w       [KB][BM]
static constexpr int GM_STAGE_XD = GM_KB * GM_BN * 4;          // f32 d_x       [KB][BN]
static constexpr int GM_STAGE = GM_STAGE_W + GM_STAGE_X + GM_STAGE_WD + GM_STAGE_XD;   // 27 KB
static_assert(GM_BM * GM_KB / 2 <= GM_THREADS, "one weight block pair per staging thread");
static_assert(GM_BN * GM_KB * 2 == 2 * GM_THREADS, "two 16-byte activation pieces per thread");
static_assert(GM_BN * GM_KB == GM_THREADS, "one d_x per thread");

__device__ __forceinline__ uint32_t nib_to_i8x4(uint32_t q, int shift) {
    const uint32_t n = (q >> shift) & 0x0F0F0F0Fu;                 // 0..15 per byte
    return ((n | 0x80808080u) - 0x08080808u) ^ 0x80808080u;      // n - 8 as int8, no cross-byte borrow
}

__device__ __forceinline__ int gm_half_off(int r, int half) {    // byte offset of a 16-B half in a 32-B row
    return r * 32 + 16 * (half ^ ((r >> 3) & 1));
}

__device__ unsigned long long g_gemm_stamps[16384 * 4];

struct GmStageRegs {
    u32x4 wa, wb;
    uint32_t wc;
    u32x4 x[2];
    float xd;
};

template <int DIAG>
__global__ __launch_bounds__(GM_THREADS, 2) void k_gemm_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes,
                                                              int nb, int M, const int8_t *__restrict__ xqs,
                                                              const float *__restrict__ xd, int N, int K,
                                                              float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave & 1, wt = wave >> 1;                        // 2 row waves x 4 token waves
    const int c = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * GM_BM;
    const int n0 = blockIdx.y * GM_BN;

    // out-of-range rows / tokens read as 0 through the descriptors' bounds
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W + (int64_t)m0 * rowbytes, (uint32_t)((int64_t)(M - m0) * rowbytes));
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(xqs + (int64_t)n0 * K, (uint32_t)((int64_t)(N - n0) * K));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(W, 0);

    // staging roles: weights (row sr, block pair sp) for tid < 128; activations (token, piece)
    // wave-uniform (readfirstlane): a per-lane descriptor choice makes hipcc wrap every buffer
    // load in a waterfall loop
    const bool wstager = __builtin_amdgcn_readfirstlane(tid >> 6) < (GM_BM * GM_KB / 2) / 64;
    const int sr = (tid >> 1) & (GM_BM - 1), sp = tid & 1;

    auto load_stage = [&](int kb0, GmStageRegs &g) {
        const bool valid = kb0 < nb && (DIAG != 3 || kb0 == 0);   // past the last stage: no traffic
        const __amdgpu_buffer_rsrc_t wr_ = (valid && wstager) ? wrs : nul;
        const int woff = (int)(sr * rowbytes) + (kb0 + 2 * sp) * Q4B;
        g.wa = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff, 0, 0);
        g.wb = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff + 16, 0, 0);
        g.wc = __builtin_amdgcn_raw_buffer_load_b32(wr_, woff + 32, 0, 0);
        const __amdgpu_buffer_rsrc_t xr_ = valid ? xrs : nul;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + GM_THREADS * i;          // 0 .. 128 tokens * 8 pieces
            const int t = idx >> 3, piece = idx & 7;       // piece: block piece>>1, half piece&1
            g.x[i] = __builtin_amdgcn_raw_buffer_load_b128(xr_, t * K + kb0 * QK + 16 * piece, 0, 0);
        }
        {
            const int b = tid >> 7, t = tid & 127;         // KB * BN == threads
            g.xd = (valid && n0 + t < N && kb0 + b < nb) ? xd[(int64_t)(n0 + t) * nb + kb0 + b] : 0.0f;
        }
    };
    auto store_stage = [&](int kb0, const GmStageRegs &g, uint8_t *st) {
        if (DIAG == 4 && kb0 > 0) {                        // diagnostic: keep the loads live, skip LDS
            asm volatile("" ::"v"(g.wa), "v"(g.wb), "v"(g.wc), "v"(g.x[0]), "v"(g.x[1]), "v"(g.xd));
            return;
        }
        uint8_t *ws = st;
        uint8_t *xs = st + GM_STAGE_W;
        float *wds = reinterpret_cast<float *>(st + GM_STAGE_W + GM_STAGE_X);
        float *xds = reinterpret_cast<float *>(st + GM_STAGE_W + GM_STAGE_X + GM_STAGE_WD);
        if (wstager) {
            // block 2sp (d = wa.x[15:0], qs = bytes 2..17) and 2sp+1 (d = wb.x[31:16], qs = wb.y..wc)
            const bool vA = kb0 + 2 * sp < nb, vB = kb0 + 2 * sp + 1 < nb;
            const uint32_t qa[4] = {__builtin_amdgcn_alignbyte(g.wa.y, g.wa.x, 2),
                                    __builtin_amdgcn_alignbyte(g.wa.z, g.wa.y, 2),
                                    __builtin_amdgcn_alignbyte(g.wa.w, g.wa.z, 2),
                                    __builtin_amdgcn_alignbyte(g.wb.x, g.wa.w, 2)};
            const uint32_t qb[4] = {g.wb.y, g.wb.z, g.wb.w, g.wc};
#pragma unroll
            for (int half = 0; half < 2; half++) {
                u32x4 ta, tb;
                ta.x = nib_to_i8x4(qa[0], 4 * half); ta.y = nib_to_i8x4(qa[1], 4 * half);
                ta.z = nib_to_i8x4(qa[2], 4 * half); ta.w = nib_to_i8x4(qa[3], 4 * half);
                tb.x = nib_to_i8x4(qb[0], 4 * half); tb.y = nib_to_i8x4(qb[1], 4 * half);
                tb.z = nib_to_i8x4(qb[2], 4 * half); tb.w = nib_to_i8x4(qb[3], 4 * half);
                *reinterpret_cast<u32x4 *>(ws + (2 * sp) * GM_BM * 32 + gm_half_off(sr, half)) = ta;
                *reinterpret_cast<u32x4 *>(ws + (2 * sp + 1) * GM_BM * 32 + gm_half_off(sr, half)) = tb;
            }
            wds[(2 * sp) * GM_BM + sr] = vA ? h2f(g.wa.x & 0xFFFFu) : 0.0f;
            wds[(2 * sp + 1) * GM_BM + sr] = vB ? h2f(g.wb.x >> 16) : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + GM_THREADS * i;
            const int t = idx >> 3, piece = idx & 7;
            *reinterpret_cast<u32x4 *>(xs + (piece >> 1) * GM_BN * 32 + gm_half_off(t, piece & 1)) = g.x[i];
        }
        xds[tid] = g.xd;
    };

    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0.0f;
    const int tok = 32 * wt + c;             // A row (token) of this lane
    const int wrow = 32 * wr + c;            // B column (weight row) of this lane

    auto compute_stage = [&](int kb0, const uint8_t *st) {
        const uint8_t *ws = st;
        const uint8_t *xs = st + GM_STAGE_W;
        const float *wds = reinterpret_cast<const float *>(st + GM_STAGE_W + GM_STAGE_X);
        const float *xds = reinterpret_cast<const float *>(st + GM_STAGE_W + GM_STAGE_X + GM_STAGE_WD);
#pragma unroll
        for (int b = 0; b < GM_KB; b++) {
            if (kb0 + b >= nb) break;
            const i32x4 af = *reinterpret_cast<const i32x4 *>(xs + b * GM_BN * 32 + gm_half_off(tok, h));
            const i32x4 bf = *reinterpret_cast<const i32x4 *>(ws + b * GM_BM * 32 + gm_half_off(wrow, h));
            const float dw = wds[b * GM_BM + wrow];
            float dx[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 f = *reinterpret_cast<const float4 *>(xds + b * GM_BN + 32 * wt + 8 * q + 4 * h);
                dx[4 * q] = f.x; dx[4 * q + 1] = f.y; dx[4 * q + 2] = f.z; dx[4 * q + 3] = f.w;
            }
            const i32x16 cz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            i32x16 cv;
            if (DIAG == 2) {                                // diagnostic: no MFMA
                cv = cz;
                cv[0] = af.x ^ bf.y;
            } else {
                cv = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, bf, cz, 0, 0, 0);
            }
            if (DIAG == 1) {                                // diagnostic: integer epilogue only
#pragma unroll
                for (int i = 0; i < 16; i++) acc[i] = __int_as_float(__float_as_int(acc[i]) + cv[i]);
                asm volatile("" ::"v"(dw), "v"(dx[0]), "v"(dx[15]));
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++) acc[i] = fmaf((float)cv[i], dw * dx[i], acc[i]);
            }
        }
    };

    // ring: LDS buffers 0/1 alternate per stage; register sets gA/gB hold stages s+1 / s+2
    // (DIAG 5: per-wave s_memtime sums of compute / staging / barrier segments)
    unsigned long long t_c = 0, t_s = 0, t_b = 0, t_mark = 0, t_begin = 0;
    auto mark = [&](unsigned long long &acc_t) {
        if (DIAG == 5) {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            acc_t += t - t_mark;
            t_mark = t;
        }
    };
    if (DIAG == 5) {
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_mark)::"memory");
        t_begin = t_mark;
    }
    const int nstages = (nb + GM_KB - 1) / GM_KB;
    GmStageRegs gA, gB;
    load_stage(0, gA);
    load_stage(GM_KB, gB);
    store_stage(0, gA, smem);
    mark(t_s);
    __syncthreads();
    mark(t_b);
    for (int s = 0; s < nstages; s += 2) {
        // even stage s in LDS buffer 0, gB holds stage s+1
        load_stage((s + 2) * GM_KB, gA);
        compute_stage(s * GM_KB, smem);
        mark(t_c);
        if (s + 1 >= nstages) break;
        store_stage((s + 1) * GM_KB, gB, smem + GM_STAGE);
        mark(t_s);
        __syncthreads();
        mark(t_b);
        // odd stage s+1 in LDS buffer 1, gA holds stage s+2
        load_stage((s + 3) * GM_KB, gB);
        compute_stage((s + 1) * GM_KB, smem + GM_STAGE);
        mark(t_c);
        if (s + 2 >= nstages) break;
        store_stage((s + 2) * GM_KB, gA, smem);
        mark(t_s);
        __syncthreads();
        mark(t_b);
    }
    if (DIAG == 5 && lane == 0) {
        const int wid = (blockIdx.y * gridDim.x + blockIdx.x) * GM_WAVES + wave;
        if (wid < 16384) {
            g_gemm_stamps[wid * 4 + 0] = t_mark - t_begin;
            g_gemm_stamps[wid * 4 + 1] = t_c;
            g_gemm_stamps[wid * 4 + 2] = t_s;
            g_gemm_stamps[wid * 4 + 3] = t_b;
        }
    }

    // epilogue: acc[i] = y[token(i)][row]; token(i) = 32wt + (i&3) + 8(i>>2) + 4h
    const int row = m0 + wrow;
    if (row < M) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int t = n0 + 32 * wt + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (t < N) y[(int64_t)t * ldy + row] = acc[i];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// GEMM v6 (default).  Same tile (64 weight rows x 128 tokens, 8 waves, one 32x32 tile per wave,
// K-stage = 4 blocks, LDS double buffer, global loads two stages ahead), restructured per block:
//   * the per-block scale d_x[token] * d_w[row] is an exact rank-1 product of two fp16 values, so
//     one v_mfma_f32_32x32x16_f16 with d_x at k = 0 of A and d_w at k = 0 of B produces all 16
//     products of a lane in the int8 tile's D layout (fp16 x fp16 is exact in fp32: the same value
//     as the CPU's fp32(d_x) * fp32(d_w)); the epilogue is cvt + fma per output and block;
//   * software pipeline over blocks: operands of block b+1 are read from LDS while block b's two
//     MFMAs run and block b-1's epilogue executes (two named result sets; the last block's
//     epilogue of a stage runs after the next stage's first MFMAs);
//   * weight staging is spread over all 512 threads (row, block, half) so that the barrier does
//     not wait on two staging waves.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Rank-1 scale product d_x (x) d_w of the prefill GEMMs: one fp16 MFMA whose A and B lanes carry a
// single nonzero half (dword 0), so every K form gives the same exact f32 products; the K = 8 form
// (v_mfma_f32_32x32x8_f16) issues in 41 nominal cycles against 51 for the K = 16 form
// (tools/gemm_mb.hip VAR 42 / 43, profiles/r03_mfma_rates.txt).  Only dword 0 of a and b may be nonzero.
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x16 scale_rank1(const u32x4 &a, const u32x4 &b) {
    const u32x2 a2 = {a.x, a.y}, b2 = {b.x, b.y};
    const f32x16 z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(half4_t, a2), __builtin_bit_cast(half4_t, b2), z, 0, 0, 0);
}
static constexpr int G6_STAGE_W = GM_KB * GM_BM * 32;           // int8 weights  [KB][BM][32]
static constexpr int G6_STAGE_X = GM_KB * GM_BN * 32;           // int8 acts     [KB][BN][32]
static constexpr int G6_STAGE_WD = GM_KB * GM_BM * 2;           // fp16 d_w      [KB][BM]
static constexpr int G6_STAGE_XD = GM_KB * GM_BN * 2;           // fp16 d_x      [KB][BN]
static constexpr int G6_STAGE = G6_STAGE_W + G6_STAGE_X + G6_STAGE_WD + G6_STAGE_XD;   // 25.5 KB
static_assert(GM_BM * GM_KB * 2 == GM_THREADS, "one (row, block, half) of the weights per thread");

struct G6Regs {
    u32x4 wa, wb;
    uint32_t wc;
    u32x4 x[2];
    float xd;
};
struct G6Ops {
    i32x4 a, b;
    uint32_t sx, sw;
};

template <int DIAG>
__global__ __launch_bounds__(GM_THREADS, 2) void k_gemm6_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes,
                                                               int nb, int M, const int8_t *__restrict__ xqs,
                                                               const float *__restrict__ xd, int N, int K,
                                                               float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave & 1, wt = wave >> 1;                        // 2 row waves x 4 token waves
    const int c = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * GM_BM;
    const int n0 = blockIdx.y * GM_BN;

    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W + (int64_t)m0 * rowbytes, (uint32_t)((int64_t)(M - m0) * rowbytes));
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(xqs + (int64_t)n0 * K, (uint32_t)((int64_t)(N - n0) * K));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(W, 0);

    // weight staging role: row sr, block sb of the stage, nibble half sh (all threads).  The 8 lanes
    // of a row are adjacent (one 72-byte span per row for the global loads).  Measured: the
    // bank-conflict-free mapping (8-lane groups = 4 rows x 2 halves) removes every LDS conflict but
    // runs 8 % slower overall (wider global footprint per wave-instruction).
    const int sr = tid >> 3, sb = (tid >> 1) & 3, sh = tid & 1;

    auto load_stage = [&](int kb0, G6Regs &g) __attribute__((always_inline)) {
        const bool valid = kb0 < nb && (DIAG != 3 || kb0 == 0);    // past the last stage: no traffic
        const __amdgpu_buffer_rsrc_t wr_ = valid ? wrs : nul;
        const int woff = (int)(sr * rowbytes) + (kb0 + (sb & ~1)) * Q4B;   // the pair holding block sb
        g.wa = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff, 0, 0);
        g.wb = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff + 16, 0, 0);
        g.wc = __builtin_amdgcn_raw_buffer_load_b32(wr_, woff + 32, 0, 0);
        const __amdgpu_buffer_rsrc_t xr_ = valid ? xrs : nul;
#pragma unroll
        for (int i = 0; i < 2; i++) {          // piece (token t, block piece>>1, half piece&1): 128 B per token
            const int idx = tid + GM_THREADS * i;
            const int t = idx >> 3, piece = idx & 7;
            g.x[i] = __builtin_amdgcn_raw_buffer_load_b128(xr_, t * K + kb0 * QK + 16 * piece, 0, 0);
        }
        {
            const int b = tid >> 7, t = tid & 127;
            g.xd = (valid && n0 + t < N && kb0 + b < nb) ? xd[(int64_t)(n0 + t) * nb + kb0 + b] : 0.0f;
        }
    };
    auto store_stage = [&](int kb0, const G6Regs &g, uint8_t *st) __attribute__((always_inline)) {
        uint8_t *ws = st;
        uint8_t *xs = st + G6_STAGE_W;
        uint16_t *wds = reinterpret_cast<uint16_t *>(st + G6_STAGE_W + G6_STAGE_X);
        uint16_t *xds = reinterpret_cast<uint16_t *>(st + G6_STAGE_W + G6_STAGE_X + G6_STAGE_WD);
        {
            const bool odd = sb & 1;
            const uint32_t q0 = odd ? g.wb.y : __builtin_amdgcn_alignbyte(g.wa.y, g.wa.x, 2);
            const uint32_t q1 = odd ? g.wb.z : __builtin_amdgcn_alignbyte(g.wa.z, g.wa.y, 2);
            const uint32_t q2 = odd ? g.wb.w : __builtin_amdgcn_alignbyte(g.wa.w, g.wa.z, 2);
            const uint32_t q3 = odd ? g.wc : __builtin_amdgcn_alignbyte(g.wb.x, g.wa.w, 2);
            u32x4 t;
            t.x = nib_to_i8x4(q0, 4 * sh); t.y = nib_to_i8x4(q1, 4 * sh);
            t.z = nib_to_i8x4(q2, 4 * sh); t.w = nib_to_i8x4(q3, 4 * sh);
            *reinterpret_cast<u32x4 *>(ws + sb * GM_BM * 32 + gm_half_off(sr, sh)) = t;
            if (sh == 0) {
                const uint32_t d16 = odd ? (g.wb.x >> 16) : (g.wa.x & 0xFFFFu);
                wds[sb * GM_BM + sr] = (uint16_t)((kb0 + sb < nb) ? d16 : 0u);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + GM_THREADS * i;
            const int t = idx >> 3, piece = idx & 7;
            *reinterpret_cast<u32x4 *>(xs + (piece >> 1) * GM_BN * 32 + gm_half_off(t, piece & 1)) = g.x[i];
        }
        xds[tid] = (uint16_t)f2h(g.xd);                            // exact: d_x is an fp16 value
    };

    const int tok = 32 * wt + c;             // A row (token) of this lane
    const int wrow = 32 * wr + c;            // B column (weight row) of this lane
    auto ld_ops = [&](const uint8_t *st, int b) __attribute__((always_inline)) {
        const uint8_t *ws = st;
        const uint8_t *xs = st + G6_STAGE_W;
        const uint16_t *wds = reinterpret_cast<const uint16_t *>(st + G6_STAGE_W + G6_STAGE_X);
        const uint16_t *xds = reinterpret_cast<const uint16_t *>(st + G6_STAGE_W + G6_STAGE_X + G6_STAGE_WD);
        G6Ops o;
        o.a = *reinterpret_cast<const i32x4 *>(xs + b * GM_BN * 32 + gm_half_off(tok, h));
        o.b = *reinterpret_cast<const i32x4 *>(ws + b * GM_BM * 32 + gm_half_off(wrow, h));
        o.sx = xds[b * GM_BN + tok];
        o.sw = wds[b * GM_BM + wrow];
        return o;
    };
    const i32x16 iz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // The int8 MFMA accumulates onto 0x4B400000, so S holds the float bits of 12582912 + sumi (exact
    // for |sumi| < 2^22; here |sumi| <= 32*8*128): float(sumi) = S_f - 12582912 exactly, a full-rate
    // v_sub_f32 instead of v_cvt_f32_i32 (compute phase -13 %; DIAG 6 keeps the cvt form)
    constexpr bool MAGIC = DIAG != 6;
    const int mg = 0x4B400000;
    const i32x16 im = {mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg};
    auto mfma2 = [&](const G6Ops &o, i32x16 &S, f32x16 &P) __attribute__((always_inline)) {
        S = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a, o.b, MAGIC ? im : iz, 0, 0, 0);
        const u32x4 as = {h == 0 ? o.sx : 0u, 0u, 0u, 0u};
        const u32x4 bs = {h == 0 ? o.sw : 0u, 0u, 0u, 0u};
        P = scale_rank1(as, bs);
    };
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0.0f;
    auto epi = [&](const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
        if (DIAG == 1) {                                            // diagnostic: no epilogue VALU
            asm volatile("" ::"v"(S[0]), "v"(S[15]), "v"(P[0]), "v"(P[15]));
            return;
        }
        if (MAGIC) {
#pragma unroll
            for (int i = 0; i < 16; i++) acc[i] = fmaf(__int_as_float(S[i]) - 12582912.0f, P[i], acc[i]);
            return;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) acc[i] = fmaf((float)S[i], P[i], acc[i]);
    };

    // one stage: blocks 0..3 from LDS buffer st; set 1 holds the previous stage's last block
    i32x16 S0, S1 = iz;
    f32x16 P0, P1 = fz;
    auto compute_stage = [&](const uint8_t *st) __attribute__((always_inline)) {
        G6Ops o0 = ld_ops(st, 0);
        G6Ops o1 = ld_ops(st, 1);
        mfma2(o0, S0, P0);
        epi(S1, P1);                          // previous stage's block 3 (zeros on the first stage)
        o0 = ld_ops(st, 2);
        mfma2(o1, S1, P1);
        epi(S0, P0);
        o1 = ld_ops(st, 3);
        mfma2(o0, S0, P0);
        epi(S1, P1);
        mfma2(o1, S1, P1);
        epi(S0, P0);
    };

    unsigned long long t_c = 0, t_s = 0, t_b = 0, t_mark = 0, t_begin = 0;
    auto mark = [&](unsigned long long &acc_t) __attribute__((always_inline)) {
        if (DIAG == 5) {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            acc_t += t - t_mark;
            t_mark = t;
        }
    };
    if (DIAG == 5) {
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_mark)::"memory");
        t_begin = t_mark;
    }
    const int nstages = (nb + GM_KB - 1) / GM_KB;
    G6Regs gA, gB;
    load_stage(0, gA);
    load_stage(GM_KB, gB);
    store_stage(0, gA, smem);
    mark(t_s);
    __syncthreads();
    mark(t_b);
    if (DIAG == 6 || DIAG == 7) {             // diagnostic: compute phase only (stage 0 data, no sync;
                                              // 6 with the cvt epilogue, 7 with the default one)
        for (int s = 0; s < nstages; s++) {
            compute_stage(smem);
            mark(t_c);
        }
    }
    for (int s = 0; DIAG != 6 && DIAG != 7 && s < nstages; s += 2) {
        load_stage((s + 2) * GM_KB, gA);
        compute_stage(smem);
        mark(t_c);
        if (s + 1 >= nstages) break;
        store_stage((s + 1) * GM_KB, gB, smem + G6_STAGE);
        mark(t_s);
        __syncthreads();
        mark(t_b);
        load_stage((s + 3) * GM_KB, gB);
        compute_stage(smem + G6_STAGE);
        mark(t_c);
        if (s + 2 >= nstages) break;
        store_stage((s + 2) * GM_KB, gA, smem);
        mark(t_s);
        __syncthreads();
        mark(t_b);
    }
    epi(S1, P1);                              // the last block
    if (DIAG == 5 && lane == 0) {
        const int wid = (blockIdx.y * gridDim.x + blockIdx.x) * GM_WAVES + wave;
        if (wid < 16384) {
            g_gemm_stamps[wid * 4 + 0] = t_mark - t_begin;
            g_gemm_stamps[wid * 4 + 1] = t_c;
            g_gemm_stamps[wid * 4 + 2] = t_s;
            g_gemm_stamps[wid * 4 + 3] = t_b;
        }
    }

    const int row = m0 + wrow;
    if (row < M) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int t = n0 + 32 * wt + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (t < N) y[(int64_t)t * ldy + row] = acc[i];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// GEMM v7: v6's tile, MFMAs and epilogue, with the activations (75 % of a stage's bytes, already
// int8) moved global -> LDS by LDS-DMA (`buffer_load_dwordx4 ... lds`, d_x by `buffer_load_dword
// ... lds`) into a 4-stage ring, so no registers hold them; the weights keep register staging
// (their nibbles are unpacked on the way into LDS) with THREE stages in flight in named register
// sets.  Per stage and thread exactly G7_OPS vector-memory operations are issued (past-the-end
// stages through zero-size descriptors), so one counted `s_waitcnt vmcnt(2*G7_OPS)` before the raw
// `s_barrier` retires stage s+1 while stages s+2 and s+3 stay in flight across it (an LDS-DMA is a
// pending LDS write on the VM counter: `__syncthreads()` would drain it).  The LDS-DMA image is
// lane-linear per wave instruction (1 KiB); the XOR half-swap of the operand reads is produced by
// choosing each lane's SOURCE address.
static constexpr int G7_NX = 4;                                  // activation ring depth (stages)
static constexpr int G7_X = GM_KB * GM_BN * 32;                  // int8 acts   [KB][BN][32]  16 KB
static constexpr int G7_XD = GM_KB * GM_BN * 2;                  // fp16 d_x    [KB][BN]       1 KB
static constexpr int G7_W = GM_KB * GM_BM * 32;                  // int8 weights [KB][BM][32]  8 KB
static constexpr int G7_WD = GM_KB * GM_BM * 2;                  // fp16 d_w    [KB][BM]
static constexpr int G7_WDZ = 2 * G7_WD;                         // zeros: the upper half-wave's d_w
static constexpr int G7_DUMMY = 256;                              // target of the zero-size d_x DMAs
static constexpr int G7_LDS = G7_NX * (G7_X + G7_XD) + 2 * (G7_W + G7_WD) + G7_WDZ + G7_DUMMY;   // 86 KB
static constexpr int G7_OPS = 3 + 2 + 1;                        // per thread per stage: W pair, 2 x glds, d_x glds
static_assert(G7_X / 1024 == 2 * GM_WAVES, "two 1-KiB activation DMA instructions per wave per stage");
static_assert(G7_XD / 256 == GM_WAVES / 2, "one 256-B d_x DMA instruction per wave of the first half per stage");

struct G7W {
    u32x4 wa, wb;
    uint32_t wc;
};

__global__ __launch_bounds__(GM_THREADS, 2) void k_gemm7_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes, int nb,
                                                               int M, const int8_t *__restrict__ xqs,
                                                               const uint16_t *__restrict__ xd16, int N, int K,
                                                               float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *xring = smem;                                          // [NX][X]
    uint16_t *xdring = reinterpret_cast<uint16_t *>(smem + G7_NX * G7_X);   // [NX][KB][BN] fp16
    uint8_t *wbuf = smem + G7_NX * (G7_X + G7_XD);                  // [2][W]
    uint16_t *wdbuf = reinterpret_cast<uint16_t *>(wbuf + 2 * G7_W);   // [2][KB][BM]
    uint16_t *wdzero = wdbuf + G7_WD;                               // [2][KB][BM] zeros
    uint8_t *dummy = reinterpret_cast<uint8_t *>(wdzero) + G7_WDZ;   // waves 4..7's d_x DMA lands here
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave & 1, wt = wave >> 1;
    const int c = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * GM_BM;
    const int n0 = blockIdx.y * GM_BN;

    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W + (int64_t)m0 * rowbytes, (uint32_t)((int64_t)(M - m0) * rowbytes));
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(xqs + (int64_t)n0 * K, (uint32_t)((int64_t)(N - n0) * K));
    // fp16 d_x, block-major [nb][Np] (quantize_q8_0_soa's copy, Np = N rounded up to 4 so that every
    // block row is dword aligned for the DMA): a block's 128 tokens are 256 bytes
    const int Np = (N + 3) & ~3;
    const __amdgpu_buffer_rsrc_t drs = make_rsrc(xd16, (uint32_t)((int64_t)nb * Np * 2));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(W, 0);
    const int sr = tid >> 3, sb = (tid >> 1) & 3, sh = tid & 1;     // weight staging role (as v6)
    if (tid < G7_WDZ / 4) reinterpret_cast<uint32_t *>(wdzero)[tid] = 0u;   // ordered by the first barrier

    // activation DMA: this wave's instructions j = 2*wave, 2*wave+1 of the stage; instruction j fills
    // LDS bytes [j KiB, (j+1) KiB) = block j/4, tokens 32*(j%4) .. +31; lane i lands at slot i =
    // (token 32*(j%4) + i/2, physical half i&1) and therefore loads logical half (i&1) ^ ((t>>3)&1)
    int xsrc[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int j = 2 * wave + q;
        const int t = 32 * (j & 3) + (lane >> 1);
        const int hh = (lane & 1) ^ ((t >> 3) & 1);
        xsrc[q] = t * K + (j >> 2) * QK + 16 * hh;                  // + kb0*32 per stage
    }
    // d_x DMA: wave w < 4 fills [block w][tokens 0 .. 127] (fp16, 2 per lane); waves 4..7 issue the
    // same instruction through the zero-size descriptor, so every wave counts 6 VM operations a stage
    const int dsrc = (wave & 3) * Np * 2 + n0 * 2 + lane * 4;       // + kb0*Np*2 per stage

    auto issue = [&](int st, G7W &g) __attribute__((always_inline)) {
        const int kb0 = st * GM_KB;
        const bool valid = kb0 < nb;                                // past the end: no traffic
#ifdef G7_NOWSTAGE
        const __amdgpu_buffer_rsrc_t wr_ = nul;        // timing diagnostic: weights cost nothing
#else
        const __amdgpu_buffer_rsrc_t wr_ = valid ? wrs : nul;
#endif
        const int woff = (int)(sr * rowbytes) + (kb0 + (sb & ~1)) * Q4B;
        g.wa = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff, 0, 0);
        g.wb = __builtin_amdgcn_raw_buffer_load_b128(wr_, woff + 16, 0, 0);
        g.wc = __builtin_amdgcn_raw_buffer_load_b32(wr_, woff + 32, 0, 0);
        const int slot = st & (G7_NX - 1);
        const __amdgpu_buffer_rsrc_t xr_ = valid ? xrs : nul;
        const __amdgpu_buffer_rsrc_t dr_ = (valid && wave < 4) ? drs : nul;
#pragma unroll
        for (int q = 0; q < 2; q++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_, (lds_void_t *)(xring + slot * G7_X + (2 * wave + q) * 1024), 16,
                                                     xsrc[q] + kb0 * QK, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            dr_, (lds_void_t *)(wave < 4 ? (uint8_t *)(xdring + slot * (G7_XD / 2) + wave * GM_BN) : dummy), 4,
            dsrc + kb0 * Np * 2, 0, 0, 0);
    };
    auto write_w = [&](int st, const G7W &g) __attribute__((always_inline)) {
#ifdef G7_NOWSTAGE
        return;
#endif
        const int kb0 = st * GM_KB;
        uint8_t *ws = wbuf + (st & 1) * G7_W;
        uint16_t *wds = wdbuf + (st & 1) * (G7_WD / 2);
        const bool odd = sb & 1;
        const uint32_t q0 = odd ? g.wb.y : __builtin_amdgcn_alignbyte(g.wa.y, g.wa.x, 2);
        const uint32_t q1 = odd ? g.wb.z : __builtin_amdgcn_alignbyte(g.wa.z, g.wa.y, 2);
        const uint32_t q2 = odd ? g.wb.w : __builtin_amdgcn_alignbyte(g.wa.w, g.wa.z, 2);
        const uint32_t q3 = odd ? g.wc : __builtin_amdgcn_alignbyte(g.wb.x, g.wa.w, 2);
        u32x4 t;
        t.x = nib_to_i8x4(q0, 4 * sh); t.y = nib_to_i8x4(q1, 4 * sh);
        t.z = nib_to_i8x4(q2, 4 * sh); t.w = nib_to_i8x4(q3, 4 * sh);
        *reinterpret_cast<u32x4 *>(ws + sb * GM_BM * 32 + gm_half_off(sr, sh)) = t;
        if (sh == 0) {
            const uint32_t d16 = odd ? (g.wb.x >> 16) : (g.wa.x & 0xFFFFu);
            wds[sb * GM_BM + sr] = (uint16_t)((kb0 + sb < nb) ? d16 : 0u);
        }
    };

    const int tok = 32 * wt + c;
    const int wrow = 32 * wr + c;
    // scale MFMA operands: every lane holds d_x at element 0 (k = 0 for h = 0, k = 8 for h = 1), the
    // weights' d_w only for h = 0 (h = 1 reads the zero region): P = d_x * d_w + d_x * 0, exact, with
    // no per-block select or conversion
    const uint16_t *wdb = h ? wdzero : wdbuf;
    auto ld_ops = [&](int st, int b) __attribute__((always_inline)) {
        const uint8_t *xs = xring + (st & (G7_NX - 1)) * G7_X;
        const uint16_t *xds = xdring + (st & (G7_NX - 1)) * (G7_XD / 2);
        const uint8_t *ws = wbuf + (st & 1) * G7_W;
        const uint16_t *wds = wdb + (st & 1) * (G7_WD / 2);
        G6Ops o;
        o.a = *reinterpret_cast<const i32x4 *>(xs + b * GM_BN * 32 + gm_half_off(tok, h));
        o.b = *reinterpret_cast<const i32x4 *>(ws + b * GM_BM * 32 + gm_half_off(wrow, h));
        o.sx = xds[b * GM_BN + tok];
        o.sw = wds[b * GM_BM + wrow];            // the upper half-wave reads zeros (see mfma2)
        return o;
    };
    const int mg = 0x4B400000;
    const i32x16 im = {mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg};
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto mfma2 = [&](const G6Ops &o, i32x16 &S, f32x16 &P) __attribute__((always_inline)) {
        S = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a, o.b, im, 0, 0, 0);
        const u32x4 as = {o.sx, 0u, 0u, 0u};
        const u32x4 bs = {o.sw, 0u, 0u, 0u};
        P = scale_rank1(as, bs);
    };
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0.0f;
    auto epi = [&](const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; i++) acc[i] = fmaf(__int_as_float(S[i]) - 12582912.0f, P[i], acc[i]);
    };
    i32x16 S0, S1 = im;
    f32x16 P1 = fz, P0;
    auto compute = [&](int st) __attribute__((always_inline)) {
#ifdef G7_IGLP
        __builtin_amdgcn_iglp_opt(G7_IGLP);      // A/B knob (tools/build_variant.sh -DG7_IGLP=0|1)
#endif
        G6Ops o0 = ld_ops(st, 0);
        G6Ops o1 = ld_ops(st, 1);
        mfma2(o0, S0, P0);
        epi(S1, P1);                          // previous stage's block 3 (S = bias, P = 0 on the first)
        o0 = ld_ops(st, 2);
        mfma2(o1, S1, P1);
        epi(S0, P0);
        o1 = ld_ops(st, 3);
        mfma2(o0, S0, P0);
        epi(S1, P1);
        mfma2(o1, S1, P1);
        epi(S0, P0);
    };
    auto sync = [&]() __attribute__((always_inline)) {   // retire stage s+1 (and the ds_writes), keep s+2, s+3
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * G7_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    };

    const int nstages = (nb + GM_KB - 1) / GM_KB;
    G7W g0, g1, g2;
    issue(0, g0);
    issue(1, g1);
    issue(2, g2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G7_OPS) : "memory");   // stage 0 landed
    write_w(0, g0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // iteration s: issue s+3 into the register set stage s used, compute s, retire s+1 + write its
    // weights, barrier.  Register sets rotate g0 -> g1 -> g2 (unrolled by 3).
    for (int s = 0; s < nstages; s += 3) {
        issue(s + 3, g0);
        compute(s);
        if (s + 1 >= nstages) break;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G7_OPS) : "memory");
        write_w(s + 1, g1);
        sync();
        issue(s + 4, g1);
        compute(s + 1);
        if (s + 2 >= nstages) break;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G7_OPS) : "memory");
        write_w(s + 2, g2);
        sync();
        issue(s + 5, g2);
        compute(s + 2);
        if (s + 3 >= nstages) break;
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G7_OPS) : "memory");
        write_w(s + 3, g0);
        sync();
    }
    epi(S1, P1);                              // the last block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may outlive the workgroup

    const int row = m0 + wrow;
    if (row < M) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int t = n0 + 32 * wt + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (t < N) y[(int64_t)t * ldy + row] = acc[i];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Prefill GEMM, round 3 (`k_gemm8_q4_0`, default for N > 128): int8-operand images DMA'd straight
// into LDS, two 32x32 output tiles per wave, the K range of every LDS stage split between the two
// halves of the workgroup.
//
// Why (tools/gemm_mb.hip, the compute phase alone with operands in LDS): per 32x32
// tile and q4_0 block the exact formulation issues an i8 MFMA, the f16 rank-1 scale MFMA and 32
// dependent VALU (acc += (S - bias) * P); on gfx950 that VALU does not overlap its own MFMAs, so the
// loop runs near the SUM of the two streams.  Two tiles per wave sharing the weight operand, with the
// scale operands carried across blocks (no per-block v_and / v_mov rebuild), is the fastest compute
// structure measured (~175 vs ~245 cycles per tile-block at two waves per SIMD for gemm7's one tile
// per wave).  M = 4096, N = 512 has only 2048 output tiles, i.e. one 2-tile wave per SIMD; the two
// workgroup halves therefore split each stage's four blocks (blocks 0-1 / 2-3) and add their partial
// tiles once at the end in a fixed order (deterministic, x -> 2x bitwise).
//
// Operands, all by LDS-DMA (`buffer_load ... lds`, no register staging, no ds_write):
//   weights: an int8 image of the q4_0 rows built per call by k_prep8_w (w = nibble - 8, exactly the
//            values the q4_0 block encodes; fp16 d copied verbatim): [M/64][nb][64 rows][32 B] with
//            the 16-byte halves of row r swapped when (r>>3)&1, so a 1 KiB DMA lands 32 rows of one
//            block in the conflict-free operand layout, + fp16 d_w [M/64][nb][64];
//   x:       the q8_0 int8 values block-major [nb][Np][32 B] (same half swap per token) + fp16 d_x
//            [nb][Np] from k_prep8_x (quantize_row_q8_0 AVX2 semantics, bit-exact, as every other
//            quantizer here).
// Every per-block integer sum stays exact (i8 MFMA, K = 32 = one block); the fp32 accumulation per
// output runs over the blocks in order within each workgroup half, the halves added at the end.
// Reference: ggml.c:11304-11351 (mul_mat_q_f32), ggml-cuda.cu:2143-2182 (dequantize + GEMM).
static constexpr int G8_BM = 64, G8_BN = 128, G8_KB = 8, G8_NS = 3, G8_LOADERS = 4;
static constexpr int G8_THREADS = (8 + G8_LOADERS) * 64;            // 8 compute waves + 4 loader waves
static constexpr int G8_W = G8_KB * G8_BM * 32;                  // int8 weights [KB][BM][32]  16 KB
static constexpr int G8_X = G8_KB * G8_BN * 32;                  // int8 x       [KB][BN][32]  32 KB
static constexpr int G8_WD = G8_KB * G8_BM * 2;                  // fp16 d_w     [KB][BM]        1 KB
static constexpr int G8_XD = G8_KB * G8_BN * 2;                  // fp16 d_x     [KB][BN]        2 KB
static constexpr int G8_STAGE = G8_W + G8_X + G8_WD + G8_XD;     // 51 KB
static constexpr int G8_ZERO = 256;                               // zeros: the upper half-wave's d_w
static constexpr int G8_LDS = G8_NS * G8_STAGE + G8_ZERO;        // 153.25 KB
static constexpr int G8_OPS = 15;                                 // DMA instructions per loader wave per stage
static_assert(G8_W / 1024 == 4 * G8_LOADERS && G8_X / 1024 == 8 * G8_LOADERS, "loader l moves blocks 2l, 2l+1");
static_assert(4 * 2 * 16 * 64 * 4 <= G8_NS * G8_STAGE, "the partial-tile exchange fits in the ring");

// x: one lane per 4 floats (8 lanes per block, k_quantize_q8_0's lane code), written block-major.
// Wave w of a workgroup takes block b = 4*blockIdx.x + w of 8 consecutive tokens (lanes 8j..8j+7 =
// token n0 + j), so its 8 image blocks are adjacent (one 256-byte store run) and each 8-lane group
// reads one 128-byte line of its token's row.  (The first version enumerated blocks along a token:
// each wave stored 8 separate 32-byte pieces Np*32 bytes apart: 7.1 -> 6.0 us mean over the bench's
// launches.  Four blocks per wave with their loads in flight together measured no faster: the launch
// is ~3 us of fixed cost + 10 MB of streaming at K = 4096.)
__global__ __launch_bounds__(256) void k_prep8_x(const float *__restrict__ x, int64_t K, int64_t N,
                                                  int8_t *__restrict__ ximg, uint16_t *__restrict__ xd16, int64_t Np) {
    const int64_t nb = K / QK;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.y * 8 + (lane >> 3);
    if (b >= nb || n >= N) return;                          // whole 8-lane groups exit together
    const int sub = lane & 7;
    const float4 v = *reinterpret_cast<const float4 *>(x + n * K + b * QK + 4 * sub);
    uint32_t d16;
    int qsum;
    const uint32_t packed = q8_block_lane(v, d16, qsum);
    const int phys = (sub >> 2) ^ (int)((n >> 3) & 1);            // 16-byte half, swapped per 8 tokens
    reinterpret_cast<uint32_t *>(ximg)[((b * Np + n) * 32 + 16 * phys + 4 * (sub & 3)) >> 2] = packed;
    if (sub == 0) xd16[b * Np + n] = (uint16_t)d16;
}

// weights: one lane per (row, block pair); a wave = 64 consecutive rows of one pair (coalesced 2 KiB
// image stores per block).  Rows >= M of the last tile are written as zeros (d = 0).
__global__ __launch_bounds__(256) void k_prep8_w(const uint8_t *__restrict__ W, int64_t rowbytes, int nb, int M,
                                                  int8_t *__restrict__ wimg, uint16_t *__restrict__ wd16) {
    const int r = threadIdx.x & 63;
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);     // (row tile, pair)
    const int npair = nb >> 1;
    const int64_t rt = item / npair;
    const int p = (int)(item - rt * npair);
    const int64_t row = rt * 64 + r;
    if (rt * 64 >= M) return;
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    uint32_t c = 0u;
    if (row < M) {
        const uint8_t *src = W + row * rowbytes + (int64_t)p * 36;
        a = *reinterpret_cast<const u32x4 *>(src);      // dword-aligned 36-byte pair (rows are 36*nb/2 B)
        b = *reinterpret_cast<const u32x4 *>(src + 16);
        c = *reinterpret_cast<const uint32_t *>(src + 32);
    }
    // block 2p: d = a.x[15:0], qs = bytes 2..17; block 2p+1: d = b.x[31:16], qs = b.y..c
    const uint32_t e[4] = {__builtin_amdgcn_alignbyte(a.y, a.x, 2), __builtin_amdgcn_alignbyte(a.z, a.y, 2),
                           __builtin_amdgcn_alignbyte(a.w, a.z, 2), __builtin_amdgcn_alignbyte(b.x, a.w, 2)};
    const uint32_t o[4] = {b.y, b.z, b.w, c};
    const int sw = (r >> 3) & 1;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t *q = k ? o : e;
        u32x4 lo, hi;                                    // elements 0..15 (low nibbles), 16..31 (high)
        lo.x = nib_to_i8x4(q[0], 0); lo.y = nib_to_i8x4(q[1], 0); lo.z = nib_to_i8x4(q[2], 0); lo.w = nib_to_i8x4(q[3], 0);
        hi.x = nib_to_i8x4(q[0], 4); hi.y = nib_to_i8x4(q[1], 4); hi.z = nib_to_i8x4(q[2], 4); hi.w = nib_to_i8x4(q[3], 4);
        if (row >= M) lo = hi = u32x4{0u, 0u, 0u, 0u};
        const int64_t blk = rt * nb + 2 * p + k;
        u32x4 *dst = reinterpret_cast<u32x4 *>(wimg + (blk * 64 + r) * 32);
        dst[sw] = lo;
        dst[sw ^ 1] = hi;
        const uint32_t d = k ? (b.x >> 16) : (a.x & 0xFFFFu);
        wd16[blk * 64 + r] = (uint16_t)(row < M ? d : 0u);
    }
}

// DIAG (timing knockouts, results invalid): 1 no compute (DMA ring + barriers only), 2 no DMA,
// 3 no DMA and no per-stage barrier (the compute loop alone)
// VAR bits (A/B knobs, all bitwise-identical results): 1 the i8 MFMA accumulates on 0 and the
// epilogue converts with v_cvt_f32_i32 (no 16-register bias operand to keep live or rebuild); 2 the
// next block's operands are read from LDS while the current block computes
template <int DIAG, int VAR = 0>
__global__ __launch_bounds__(G8_THREADS, 1) void k_gemm8_q4_0(const int8_t *__restrict__ wimg,
                                                               const uint16_t *__restrict__ wd16, int nb, int M,
                                                               const int8_t *__restrict__ ximg,
                                                               const uint16_t *__restrict__ xd16, int64_t Np, int N,
                                                               float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *zero = smem + G8_NS * G8_STAGE;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
    const int rt = blockIdx.x;
    const int m0 = rt * G8_BM, n0 = blockIdx.y * G8_BN;
    if (tid < G8_ZERO / 4) reinterpret_cast<uint32_t *>(zero)[tid] = 0u;   // ordered by the first barrier

    // descriptors: this row tile's slice of the weight image, the whole x image
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(wimg + (int64_t)rt * nb * 2048, (uint32_t)nb * 2048u);
    const __amdgpu_buffer_rsrc_t wdrs = make_rsrc(wd16 + (int64_t)rt * nb * 64, (uint32_t)nb * 128u);
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(ximg, (uint32_t)((int64_t)nb * Np * 32));
    const __amdgpu_buffer_rsrc_t xdrs = make_rsrc(xd16, (uint32_t)((int64_t)nb * Np * 2));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(wimg, 0);

    // DMA roles: loader wave l = wave - 8 moves blocks 2l, 2l+1 of every stage: weights (2 x 1 KiB
    // each), x (4 x 1 KiB each), d_x (256 B each), d_w (both blocks in one 256-B instruction) = 15
    // instructions; the compute waves issue none (an LDS-DMA costs its issuing wave 60-185 cycles,
    // MI355X_MICROARCH.md cycle constants, which measured as unhidden time in the compute waves)
    const int lw = wave - 8;
    const int lb = 2 * lw;                                                         // first block
    auto issue = [&](int st) __attribute__((always_inline)) {
        if (DIAG >= 2 || wave < 8) return;
        uint8_t *base = smem + (st % G8_NS) * G8_STAGE;
        const int kb0 = st * G8_KB;
        const bool v = kb0 + lb < nb;                                             // nb even: both or none
        const __amdgpu_buffer_rsrc_t wr_ = v ? wrs : nul, xr_ = v ? xrs : nul, dr_ = v ? xdrs : nul,
                                     wdr_ = v ? wdrs : nul;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = lb + j;
#pragma unroll
            for (int r = 0; r < 2; r++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr_, (lds_void_t *)(base + b * 2048 + r * 1024), 16,
                                                         (kb0 + b) * 2048 + r * 1024 + lane * 16, 0, 0, 0);
            const int xs = (int)(((int64_t)(kb0 + b) * Np + n0) * 32) + lane * 16;
#pragma unroll
            for (int r = 0; r < 4; r++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_, (lds_void_t *)(base + G8_W + b * 4096 + r * 1024), 16,
                                                         xs + r * 1024, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr_, (lds_void_t *)(base + G8_W + G8_X + G8_WD + b * 256), 4,
                                                     (int)(((int64_t)(kb0 + b) * Np + n0) * 2) + lane * 4, 0, 0, 0);
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wdr_, (lds_void_t *)(base + G8_W + G8_X + lb * 128), 4,
                                                 (kb0 + lb) * 128 + lane * 4, 0, 0, 0);
    };

    // compute roles: workgroup half g takes blocks 4g .. 4g+3 of every stage; wave q of the half owns
    // weight rows 32*(q&1)..+31 and token tiles 64*(q>>1) + {0, 32}
    const int g = (wave >> 2) & 1, q = wave & 3;          // (loader waves: unused)
    const int wrow = 32 * (q & 1) + c;
    const int t0 = 64 * (q >> 1) + c, t1 = t0 + 32;
    const int hw = 16 * (h ^ ((wrow >> 3) & 1));
    const int h0 = 16 * (h ^ ((t0 >> 3) & 1)), h1 = 16 * (h ^ ((t1 >> 3) & 1));
    constexpr bool CVT = VAR & 1, PF = VAR & 2, GRP = VAR & 4, STAG = VAR & 8, PRIO = VAR & 16;
    const int mg = CVT ? 0 : 0x4B400000;
    const i32x16 im = {mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg};
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float acc0[16], acc1[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.0f;
    i32x16 S0 = im, S1 = im;
    f32x16 P0 = fz, P1 = fz;
    // scale operands, carried: only element 0 (k = 0 / k = 8) is rewritten per block; the upper
    // half-wave's d_w comes from the zero region, so P = d_x * d_w exactly
    u32x4 as0 = {0u, 0u, 0u, 0u}, as1 = {0u, 0u, 0u, 0u}, bs = {0u, 0u, 0u, 0u};
    auto epi = [&](float *a, const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; i++)
            a[i] = fmaf(CVT ? (float)S[i] : __int_as_float(S[i]) - 12582912.0f, P[i], a[i]);
    };
    struct Ops {
        i32x4 bw, a0, a1;
        uint32_t sw, sx0, sx1;
    };
    auto rd = [&](int st, int b) __attribute__((always_inline)) {
        const uint8_t *base = smem + (st % G8_NS) * G8_STAGE;
        Ops o;
        o.bw = *reinterpret_cast<const i32x4 *>(base + b * 2048 + wrow * 32 + hw);
        o.a0 = *reinterpret_cast<const i32x4 *>(base + G8_W + b * 4096 + t0 * 32 + h0);
        o.a1 = *reinterpret_cast<const i32x4 *>(base + G8_W + b * 4096 + t1 * 32 + h1);
        o.sw = *reinterpret_cast<const uint16_t *>((h ? zero : base + G8_W + G8_X + b * 128) + wrow * 2);
        const uint16_t *xd = reinterpret_cast<const uint16_t *>(base + G8_W + G8_X + G8_WD + b * 256);
        o.sx0 = xd[t0];
        o.sx1 = xd[t1];
        return o;
    };
    auto block = [&](const Ops &o) __attribute__((always_inline)) {
        bs.x = o.sw;
        as0.x = o.sx0;
        as1.x = o.sx1;
        if constexpr (GRP) {
            // the block's four MFMAs back to back, then both epilogues: the wave parks on the matrix pipe
            // while its SIMD partner runs its VALU (the two compute waves of a SIMD fall out of phase);
            // every epilogue reads MFMA results issued a whole burst earlier
            epi(acc0, S0, P0);
            epi(acc1, S1, P1);
            __builtin_amdgcn_sched_barrier(0);
            S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a0, o.bw, im, 0, 0, 0);
            P0 = scale_rank1(as0, bs);
            S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a1, o.bw, im, 0, 0, 0);
            P1 = scale_rank1(as1, bs);
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
        S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a0, o.bw, im, 0, 0, 0);
        P0 = scale_rank1(as0, bs);
        epi(acc1, S1, P1);                     // tile 1 of the previous block (S1 = bias, P1 = 0 at first)
        S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(o.a1, o.bw, im, 0, 0, 0);
        P1 = scale_rank1(as1, bs);
        epi(acc0, S0, P0);
    };
    auto sync = [&]() __attribute__((always_inline)) {   // retire stage s+1, keep s+2 in flight
        if (DIAG == 3) return;
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((G8_NS - 2) * G8_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    };

    const int nstages = (nb + G8_KB - 1) / G8_KB;
    // STAG: the second compute half starts every stage half a block late, so that one wave of each SIMD
    // is in its MFMA burst while its partner runs VALU (MI355X_MICROARCH.md, two waves per SIMD item 9);
    // PRIO: that half at priority 1 (item 4)
    if (PRIO && wave >= 4 && wave < 8) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < G8_NS - 1; st++) issue(st);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((G8_NS - 2) * G8_OPS) : "memory");   // stage 0 landed
    __builtin_amdgcn_s_barrier();
    for (int s = 0; s < nstages; s++) {
        issue(s + G8_NS - 1);
        const int kb = s * G8_KB + 4 * g;
        if (STAG && g == 1 && wave < 8) __builtin_amdgcn_s_sleep(2);
        if (DIAG != 1 && wave < 8) {
            if (PF) {                              // nb is even and kb too: blocks come in valid pairs
                Ops o = rd(s, 4 * g);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (kb + j >= nb) break;
                    Ops n = o;
                    if (j < 3) n = rd(s, 4 * g + j + 1);
                    block(o);
                    o = n;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (kb + j < nb) block(rd(s, 4 * g + j));
            }
        }
        sync();
    }
    if (GRP) epi(acc0, S0, P0);
    epi(acc1, S1, P1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may outlive the ring
    __syncthreads();
    // the halves' partial tiles: half 1 -> LDS, half 0 adds (acc_half0 + acc_half1, fixed order)
    float *red = reinterpret_cast<float *>(smem);
    if (wave >= 4 && wave < 8) {
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            *reinterpret_cast<float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4) = {acc0[i], acc0[i + 1], acc0[i + 2], acc0[i + 3]};
            *reinterpret_cast<float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4) = {acc1[i], acc1[i + 1], acc1[i + 2], acc1[i + 3]};
        }
    }
    __syncthreads();
    if (wave < 4) {
        const int row = m0 + wrow;
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            const float4 o0 = *reinterpret_cast<const float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4);
            const float4 o1 = *reinterpret_cast<const float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4);
            acc0[i] += o0.x; acc0[i + 1] += o0.y; acc0[i + 2] += o0.z; acc0[i + 3] += o0.w;
            acc1[i] += o1.x; acc1[i + 1] += o1.y; acc1[i + 2] += o1.z; acc1[i + 3] += o1.w;
        }
        if (row < M) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int tk = n0 + 64 * (q >> 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (tk < N) y[(int64_t)tk * ldy + row] = acc0[i];
                if (tk + 32 < N) y[(int64_t)(tk + 32) * ldy + row] = acc1[i];
            }
        }
    }
}

int64_t gemm8_np(int64_t N) { return (N + 3) & ~(int64_t)3; }
size_t gemm8_x_bytes(int64_t K, int64_t N) { return (size_t)(K / QK) * gemm8_np(N) * 34; }
size_t gemm8_w_bytes(int64_t K, int64_t M) { return (size_t)((M + 63) / 64) * (K / QK) * 64 * 34; }

hipError_t gemm8_prep_x(const float *x, int64_t K, int64_t N, void *xws, hipStream_t s) {
    const int64_t nb = K / QK;
    if (N <= 0 || nb <= 0) return hipSuccess;
    if ((N + 7) / 8 > 65535) return hipErrorInvalidValue;          // grid.y limit
    const int64_t Np = gemm8_np(N);
    int8_t *ximg = (int8_t *)xws;
    uint16_t *xd16 = (uint16_t *)((char *)xws + (size_t)nb * Np * 32);
    (void)hipGetLastError();
    launch_k(k_prep8_x, dim3((unsigned)((nb + 3) / 4), (unsigned)((N + 7) / 8)), dim3(256), 0, s, x, K, N, ximg, xd16, Np);
    return hipGetLastError();
}

hipError_t gemm8_prep_w(const void *W, int64_t K, int64_t M, void *wws, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t Mt = (M + 63) / 64;
    int8_t *wimg = (int8_t *)wws;
    uint16_t *wd16 = (uint16_t *)((char *)wws + (size_t)Mt * nb * 2048);
    (void)hipGetLastError();
    const int64_t items = Mt * (nb / 2);                  // (row tile, pair) items, 4 per 256-thread block
    launch_k(k_prep8_w, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, (const uint8_t *)W, (int64_t)nb * Q4B, nb,
             (int)M, wimg, wd16);
    return hipGetLastError();
}

hipError_t gemm8_run(const void *wws, int64_t K, int64_t M, const void *xws, int64_t N, float *y, int64_t ldy,
                     hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t Mt = (M + 63) / 64, Np = gemm8_np(N);
    const int8_t *wimg = (const int8_t *)wws;
    const uint16_t *wd16 = (const uint16_t *)((const char *)wws + (size_t)Mt * nb * 2048);
    const int8_t *ximg = (const int8_t *)xws;
    const uint16_t *xd16 = (const uint16_t *)((const char *)xws + (size_t)nb * Np * 32);
    if ((int64_t)nb * Np * 32 >= ((int64_t)1 << 31) || (int64_t)nb * 2048 >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        for (auto k : {k_gemm8_q4_0<0, 0>, k_gemm8_q4_0<0, 1>, k_gemm8_q4_0<0, 2>, k_gemm8_q4_0<0, 3>, k_gemm8_q4_0<0, 7>,
                       k_gemm8_q4_0<0, 15>, k_gemm8_q4_0<0, 23>, k_gemm8_q4_0<0, 31>,
                       k_gemm8_q4_0<3, 7>,
                       k_gemm8_q4_0<1, 3>, k_gemm8_q4_0<2, 3>, k_gemm8_q4_0<3, 3>}) {
            hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS);
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
    // GGML_HIP_GEMM8_VAR (A/B, tools/r3_g8var.sh, kernel medians at 4096x4096x512): 0 33.3 us, 3 = cvt
    // epilogue + operand prefetch 29.6-29.8, 7 = 3 + MFMA bursts 29.2-29.4 (default; compute-only knockout
    // 25.0 -> 23.8); GGML_HIP_GEMM_DIAG 81 / 82 / 83 = DMA-only / no DMA / no DMA and no barrier
    static const int diag = env_int("GGML_HIP_GEMM_DIAG", 0);
    static const int var = env_int("GGML_HIP_GEMM8_VAR", 7);
    auto kern = diag == 81 ? k_gemm8_q4_0<1, 3> : diag == 82 ? k_gemm8_q4_0<2, 3> : diag == 83 ? k_gemm8_q4_0<3, 3>
              : diag == 87 ? k_gemm8_q4_0<3, 7> : var == 3 ? k_gemm8_q4_0<0, 3> : var == 15 ? k_gemm8_q4_0<0, 15>
              : var == 23 ? k_gemm8_q4_0<0, 23> : var == 31 ? k_gemm8_q4_0<0, 31>
              : var == 0 ? k_gemm8_q4_0<0, 0> : var == 1 ? k_gemm8_q4_0<0, 1> : var == 2 ? k_gemm8_q4_0<0, 2>
              : k_gemm8_q4_0<0, 7>;
    (void)hipGetLastError();
    launch_k(kern, dim3((unsigned)Mt, (unsigned)((N + G8_BN - 1) / G8_BN)), dim3(G8_THREADS), G8_LDS, s, wimg, wd16,
             nb, (int)M, ximg, xd16, Np, (int)N, y, ldy);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Prefill GEMM v9: the exact per-block integer sum on the block-scaled fp6 matrix cores
// (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 operands, tools/fp6_check.hip: 0 mismatches over 262k
// outputs).  Why: gemm8's compute phase is bound by its epilogue, which first converts each i8
// MFMA's int32 block sums to float (16 VALU per tile and block) before the scale fma; the fp6
// instruction returns the same integer already as an f32 (every partial sum an integer < 2^24, so
// exact), which leaves the epilogue one fma per output (tools/gemm_mb.hip VAR36 vs VAR21: 172 vs 210
// cycles per tile-block on the same box, although the fp6 instruction takes twice the i8 one's cycles).
// Operand encoding (every value exact in e2m3 = 1 sign, 2 exponent, 3 mantissa bits, |v| <= 7.5):
//   weights  w = nibble - 8 in [-8, 7] as w/2, block scale 2^1, in both K halves of the instruction;
//   x        the q8_0 value q in [-128, 127] split as q = 16*(q >> 4) + (q & 15): K half 0 holds
//            (q >> 4)/2 with scale 2^5, K half 1 holds (q & 15)/2 with scale 2^1,
// so one 32x32x64 instruction = sum_k w*16*(q >> 4) + w*(q & 15) = sum_k w*q, the block's sumi.
// The epilogue acc = fma(S, d_x*d_w, acc) gives bit for bit gemm8's values (same integer, same scale
// product, same block order and workgroup-half split).
// Images (32 codes x 6 bits = 24 B per row and block, element j at bits 6j..6j+5, stored as a 16-byte
// and an 8-byte part so that every operand read is one ds_read_b128 + one ds_read_b64 on 16/8-byte
// strides, bank-conflict free): weights [M/128][nb][128 rows x 16 B | 128 rows x 8 B] + fp16 d_w
// [M/128][nb][128] (26 B per 32 weights: 1.44x the q4_0 bytes); x [nb][3][Np][16 B]: part 0 = the
// first 16 B of the (q >> 4) codes, part 1 = those of the (q & 15) codes, part 2 = the last 8 B of
// both (swapped for tokens with bit 4 set: the b64 reads of a half-wave cover all 64 banks) + fp16
// d_x [nb][Np].
// Tile 128 weight rows x 64 tokens (the stage is 51 KB like gemm8's, ring of 3); wave q of half g
// owns tokens 32(q&1).. and rows 64(q>>1) + {0, 32} (the x operand shared by its two tiles).
static constexpr int G9_BM = 128, G9_BN = 64, G9_KB = 8, G9_NS = 3, G9_LOADERS = 4;
static constexpr int G9_THREADS = (8 + G9_LOADERS) * 64;
static constexpr int G9_WB = G9_BM * 24;                          // weight codes per block   3 KB
static constexpr int G9_XB = G9_BN * 48;                          // x codes per block        3 KB
static constexpr int G9_W = G9_KB * G9_WB;                        // 24 KB
static constexpr int G9_X = G9_KB * G9_XB;                        // 24 KB
static constexpr int G9_WD = G9_KB * G9_BM * 2;                   // fp16 d_w                 2 KB
static constexpr int G9_XD = G9_KB * G9_BN * 2;                   // fp16 d_x                 1 KB
static constexpr int G9_STAGE = G9_W + G9_X + G9_WD + G9_XD;      // 51 KB
static constexpr int G9_ZERO = 1024;                               // zero d_w for the h = 1 lanes
static constexpr int G9_LDS = G9_NS * G9_STAGE + G9_ZERO;         // 154 KB
static constexpr int G9_OPS = 15;                                  // DMA instructions per loader wave per stage
static_assert(G9_WB == 3 * 1024 && G9_XB == 3 * 1024, "3 x 1 KiB DMAs per block and operand");
static_assert(4 * 2 * 16 * 64 * 4 <= G9_NS * G9_STAGE, "the partial-tile exchange fits in the ring");
static constexpr int G9_SCALE_1 = 128, G9_SCALE_5 = 132;           // E8M0 block scales 2^1, 2^5

typedef int i32x8 __attribute__((ext_vector_type(8)));

// e2m3 code of n/2 for an integer n in [-15, 15]
// (branch-free: with e = (a >= 4) + (a >= 8), c = (a << (2 - e)) + 8e is 4a / 8 + 2a / 16 + a)
__device__ __forceinline__ uint32_t e2m3_half(int n) {
    const uint32_t a = (uint32_t)__builtin_abs(n);
    const uint32_t e = (uint32_t)(a >= 4u) + (uint32_t)(a >= 8u);
    return ((uint32_t)n >> 26 & 0x20u) | ((a << (2u - e)) + 8u * e);
}
// four 6-bit codes (elements 4m .. 4m+3) as one 24-bit field
__device__ __forceinline__ uint32_t f6x4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    return c0 | (c1 << 6) | (c2 << 12) | (c3 << 18);
}
// 32 codes = fields F0..F7 (24 bits each) -> 6 dwords, element j at bits 6j..6j+5
__device__ __forceinline__ void f6_pack(const uint32_t *F, uint32_t *D) {
    D[0] = F[0] | (F[1] << 24);
    D[1] = (F[1] >> 8) | (F[2] << 16);
    D[2] = (F[2] >> 16) | (F[3] << 8);
    D[3] = F[4] | (F[5] << 24);
    D[4] = (F[5] >> 8) | (F[6] << 16);
    D[5] = (F[6] >> 16) | (F[7] << 8);
}

// x: the q8_0 lane code of k_prep8_x (8 lanes per block, wave = 8 tokens of one block); each lane's
// four q give four (q >> 4) and four (q & 15) codes (24 bits each), and lanes 0-5 of the group
// assemble the block's six dwords of each half from their neighbours' fields.
template <bool DPP>
__global__ __launch_bounds__(256) void k_prep9_x(const float *__restrict__ x, int64_t K, int64_t N,
                                                  uint8_t *__restrict__ ximg, uint16_t *__restrict__ xd16, int64_t Np) {
    const int64_t nb = K / QK;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.y * 8 + (lane >> 3);
    if (b >= nb) return;                                    // wave-uniform
    const bool live = n < N;
    const int sub = lane & 7;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (live) v = *reinterpret_cast<const float4 *>(x + n * K + b * QK + 4 * sub);
    uint32_t d16;
    int qsum;
    const uint32_t packed = q8_block_lane(v, d16, qsum);
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int q = (int)(int8_t)(packed >> (8 * e));
        hi[e] = e2m3_half(q >> 4);
        lo[e] = e2m3_half(q & 15);
    }
    const uint32_t Fh = f6x4(hi[0], hi[1], hi[2], hi[3]), Fl = f6x4(lo[0], lo[1], lo[2], lo[3]);
    // dword k of a half: fields s and s + 1 shifted by off (k = 0..5 -> (s, off) = (0,0) (1,8) (2,16)
    // (4,0) (5,8) (6,16))
    const int k = sub < 6 ? sub : 5;
    const int off = 8 * (k % 3);
    // the fields of lanes +1 and +2 by DPP row shifts (groups of 8 lanes sit inside 16-lane rows; lanes
    // 6 and 7, which read past their group, store nothing): k < 3 takes fields (own, +1), k >= 3 (+1, +2)
    // (DPP false: the same fields through __shfl, the round-3 first version; A/B GGML_HIP_PREP9_DPP=0)
    const int base = lane & ~7, s1 = base + (k < 3 ? k : k + 1);
    const uint32_t Fh1 = DPP ? (uint32_t)__builtin_amdgcn_mov_dpp((int)Fh, 0x101, 0xF, 0xF, false)   // row_shl:1
                             : (uint32_t)__shfl((int)Fh, base + k + 1);
    const uint32_t Fh2 = DPP ? (uint32_t)__builtin_amdgcn_mov_dpp((int)Fh, 0x102, 0xF, 0xF, false)   // row_shl:2
                             : (uint32_t)__shfl((int)Fh, s1 + 1);
    const uint32_t Fl1 = DPP ? (uint32_t)__builtin_amdgcn_mov_dpp((int)Fl, 0x101, 0xF, 0xF, false)
                             : (uint32_t)__shfl((int)Fl, base + k + 1);
    const uint32_t Fl2 = DPP ? (uint32_t)__builtin_amdgcn_mov_dpp((int)Fl, 0x102, 0xF, 0xF, false)
                             : (uint32_t)__shfl((int)Fl, s1 + 1);
    const bool lo3 = k < 3;
    const uint32_t h0 = lo3 ? Fh : Fh1, h1 = lo3 ? Fh1 : Fh2;
    const uint32_t l0 = lo3 ? Fl : Fl1, l1 = lo3 ? Fl1 : Fl2;
    if (!live || sub >= 6) return;
    const uint32_t dh = (h0 >> off) | (h1 << (24 - off)), dl = (l0 >> off) | (l1 << (24 - off));
    const int sw = (int)((n >> 4) & 1);
    uint32_t *p0 = reinterpret_cast<uint32_t *>(ximg + ((b * 3 + 0) * Np + n) * 16);
    uint32_t *p1 = reinterpret_cast<uint32_t *>(ximg + ((b * 3 + 1) * Np + n) * 16);
    uint32_t *p2 = reinterpret_cast<uint32_t *>(ximg + ((b * 3 + 2) * Np + n) * 16);
    if (k < 4) {
        p0[k] = dh;
        p1[k] = dl;
    } else {
        p2[2 * sw + k - 4] = dh;
        p2[2 * (sw ^ 1) + k - 4] = dl;
    }
    if (sub == 0) xd16[b * Np + n] = (uint16_t)d16;
}

// weights: one lane per (row, block pair), 128 consecutive rows of one pair per 128 lanes; rows >= M
// of the last tile are zeros (d = 0)
__global__ __launch_bounds__(256) void k_prep9_w(const uint8_t *__restrict__ W, int64_t rowbytes, int nb, int M,
                                                  uint8_t *__restrict__ wimg, uint16_t *__restrict__ wd16) {
    const int r = threadIdx.x & 127;
    const int64_t item = (int64_t)blockIdx.x * 2 + (threadIdx.x >> 7);     // (row tile, pair)
    const int npair = nb >> 1;
    const int64_t rt = item / npair;
    const int p = (int)(item - rt * npair);
    const int64_t row = rt * 128 + r;
    if (rt * 128 >= M) return;
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    uint32_t c = 0u;
    const bool live = row < M;
    if (live) {
        const uint8_t *src = W + row * rowbytes + (int64_t)p * 36;
        a = *reinterpret_cast<const u32x4 *>(src);
        b = *reinterpret_cast<const u32x4 *>(src + 16);
        c = *reinterpret_cast<const uint32_t *>(src + 32);
    }
    const uint32_t e[4] = {__builtin_amdgcn_alignbyte(a.y, a.x, 2), __builtin_amdgcn_alignbyte(a.z, a.y, 2),
                           __builtin_amdgcn_alignbyte(a.w, a.z, 2), __builtin_amdgcn_alignbyte(b.x, a.w, 2)};
    const uint32_t o[4] = {b.y, b.z, b.w, c};
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
        const uint32_t *q = kk ? o : e;
        uint32_t F[8];
#pragma unroll
        for (int m = 0; m < 8; m++) {                   // elements 4m..4m+3: m < 4 low nibbles, else high
            const uint32_t word = q[m & 3], sh = m < 4 ? 0u : 4u;
            uint32_t cc[4];
#pragma unroll
            for (int t = 0; t < 4; t++) cc[t] = live ? e2m3_half((int)((word >> (8 * t + sh)) & 15u) - 8) : 0u;
            F[m] = f6x4(cc[0], cc[1], cc[2], cc[3]);
        }
        uint32_t D[6];
        f6_pack(F, D);
        const int64_t blk = rt * nb + 2 * p + kk;
        *reinterpret_cast<u32x4 *>(wimg + blk * G9_WB + r * 16) = u32x4{D[0], D[1], D[2], D[3]};
        *reinterpret_cast<u32x2 *>(wimg + blk * G9_WB + 2048 + r * 8) = u32x2{D[4], D[5]};
        const uint32_t d = kk ? (b.x >> 16) : (a.x & 0xFFFFu);
        wd16[blk * 128 + r] = (uint16_t)(live ? d : 0u);
    }
}

// DIAG (timing knockouts, results invalid): 1 no compute, 2 no DMA, 3 no DMA and no barrier, 4 / 5 no
// x / no weight DMA (the other operand still streams)
// VAR bits (A/B knobs, bitwise-identical results): 1 operands read right before their block (no
// prefetch), 2 packed f32 epilogue (v_pk_fma_f32), 4 two named operand sets read one block ahead
// (ping-pong, no copies), 8 loader waves stage through registers (buffer_load_dwordx4 -> ds_write_b128)
// instead of LDS-DMA, 16 the scale product on the K = 8 fp16 MFMA, 32 (with 1) per-stage VGPR address
// bases with the block offsets as ds_read immediates (no address VALU per block; a variant that also
// read the next block's operands before the current block needed 168 VGPRs and spilled 81: dropped),
// 128 loader waves at s_setprio 3, 256 the burst as fp6, fp6, fp16, fp16
// Tile list of one launch: the row tiles of 1..4 sibling matrices sharing x (wq|wk|wv, w1|w3), tb[i]
// = first row tile of matrix i, then the token tiles of each row tile.  Tile order (`xcd`):
// 0 = row tile fastest (workgroup id = rt + Mt*ty: the token tiles of a row tile land on XCD
// (rt + Mt*ty) % 8, i.e. on one XCD only when Mt % 8 == 0), 1 = XCD-aware: the hardware deals
// workgroup ids round robin to the 8 XCDs, so id i runs on XCD i % 8; tile j = (i % 8)*C + i/8 (C =
// G/8) gives XCD x the contiguous tile range [xC, xC + C) in row-tile-major order: the Ny token tiles
// of a row tile run on one XCD, together, and its weight image is fetched into one L2 only.
struct G9Mats {
    const uint8_t *wimg[4];
    const uint16_t *wd16[4];
    float *y[4];
    int64_t ldy[4];
    int M[4];
    int tb[5];
    int n, ny, xcd;
};

template <int DIAG, int VAR = 0>
__global__ __launch_bounds__(G9_THREADS, 1) void k_gemm9_q4_0(const G9Mats mats, int nb,
                                                               const uint8_t *__restrict__ ximg,
                                                               const uint16_t *__restrict__ xd16, int64_t Np, int N) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *zero = smem + G9_NS * G9_STAGE;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
    const int G = (int)gridDim.x, Mt = mats.tb[mats.n];
    int j = (int)blockIdx.x;
    if (mats.xcd) {
        const int C = G >> 3;
        if (j < 8 * C) j = (j & 7) * C + (j >> 3);
    }
    const int rtg = mats.xcd ? j / mats.ny : j % Mt, ty = mats.xcd ? j - rtg * mats.ny : j / Mt;
    // matrix of row tile rtg (selects, no dynamic kernarg indexing)
    const int mi = (mats.n > 1 && rtg >= mats.tb[1]) + (mats.n > 2 && rtg >= mats.tb[2]) + (mats.n > 3 && rtg >= mats.tb[3]);
    const uint8_t *wimg = mi == 0 ? mats.wimg[0] : mi == 1 ? mats.wimg[1] : mi == 2 ? mats.wimg[2] : mats.wimg[3];
    const uint16_t *wd16 = mi == 0 ? mats.wd16[0] : mi == 1 ? mats.wd16[1] : mi == 2 ? mats.wd16[2] : mats.wd16[3];
    float *y = mi == 0 ? mats.y[0] : mi == 1 ? mats.y[1] : mi == 2 ? mats.y[2] : mats.y[3];
    const int64_t ldy = mi == 0 ? mats.ldy[0] : mi == 1 ? mats.ldy[1] : mi == 2 ? mats.ldy[2] : mats.ldy[3];
    const int M = mi == 0 ? mats.M[0] : mi == 1 ? mats.M[1] : mi == 2 ? mats.M[2] : mats.M[3];
    const int rt = rtg - (mi == 0 ? 0 : mi == 1 ? mats.tb[1] : mi == 2 ? mats.tb[2] : mats.tb[3]);
    const int m0 = rt * G9_BM, n0 = ty * G9_BN;
    if (tid < G9_ZERO / 4) reinterpret_cast<uint32_t *>(zero)[tid] = 0u;

    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(wimg + (int64_t)rt * nb * G9_WB, (uint32_t)nb * G9_WB);
    const __amdgpu_buffer_rsrc_t wdrs = make_rsrc(wd16 + (int64_t)rt * nb * G9_BM, (uint32_t)nb * G9_BM * 2u);
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(ximg, (uint32_t)((int64_t)nb * Np * 48));
    const __amdgpu_buffer_rsrc_t xdrs = make_rsrc(xd16, (uint32_t)((int64_t)nb * Np * 2));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(wimg, 0);

    // loader wave l = wave - 8 moves blocks 2l, 2l+1 of every stage: weights and x 3 x 1 KiB each per
    // block, d_w 256 B per block, d_x of both blocks in one instruction (lanes 32-63: the second) = 15
    const int lw = wave - 8;
    const int lb = 2 * lw;
    auto issue = [&](int st) __attribute__((always_inline)) {
        if ((DIAG >= 2 && DIAG <= 3) || wave < 8) return;
        uint8_t *base = smem + (st % G9_NS) * G9_STAGE;
        const int kb0 = st * G9_KB;
        const bool v = kb0 + lb < nb;                                             // nb even: both or none
        const __amdgpu_buffer_rsrc_t wr_ = v && DIAG != 5 ? wrs : nul, xr_ = v && DIAG != 4 ? xrs : nul,
                                     dr_ = v ? xdrs : nul, wdr_ = v ? wdrs : nul;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = lb + j;
#pragma unroll
            for (int r = 0; r < 3; r++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr_, (lds_void_t *)(base + b * G9_WB + r * 1024), 16,
                                                         (kb0 + b) * G9_WB + r * 1024 + lane * 16, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 3; r++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_, (lds_void_t *)(base + G9_W + b * G9_XB + r * 1024), 16,
                                                         (int)((((int64_t)(kb0 + b) * 3 + r) * Np + n0) * 16) + lane * 16,
                                                         0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wdr_, (lds_void_t *)(base + G9_W + G9_X + b * 256), 4,
                                                     (kb0 + b) * 256 + lane * 4, 0, 0, 0);
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dr_, (lds_void_t *)(base + G9_W + G9_X + G9_WD + lb * 128), 4,
                                                 (int)(((int64_t)(kb0 + lb + h) * Np + n0) * 2) + c * 4, 0, 0, 0);
    };
    // VAR & 8: the same bytes through the loader waves' registers (loaded one stage ahead of the write)
    u32x4 stg[12];
    uint32_t stg_dw[2], stg_dx = 0u;
    auto load_regs = [&](int st) __attribute__((always_inline)) {
        if (DIAG >= 2 || wave < 8) return;
        const int kb0 = st * G9_KB;
        const bool v = kb0 + lb < nb;
        const __amdgpu_buffer_rsrc_t wr_ = v ? wrs : nul, xr_ = v ? xrs : nul, dr_ = v ? xdrs : nul,
                                     wdr_ = v ? wdrs : nul;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = lb + j;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                stg[6 * j + r] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                               wr_, (kb0 + b) * G9_WB + r * 1024 + lane * 16, 0, 0));
                stg[6 * j + 3 + r] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                               xr_, (int)((((int64_t)(kb0 + b) * 3 + r) * Np + n0) * 16) + lane * 16, 0, 0));
            }
            stg_dw[j] = __builtin_amdgcn_raw_buffer_load_b32(wdr_, (kb0 + b) * 256 + lane * 4, 0, 0);
        }
        stg_dx = __builtin_amdgcn_raw_buffer_load_b32(dr_, (int)(((int64_t)(kb0 + lb + h) * Np + n0) * 2) + c * 4, 0, 0);
    };
    auto store_regs = [&](int st) __attribute__((always_inline)) {
        if (DIAG >= 2 || wave < 8) return;
        uint8_t *base = smem + (st % G9_NS) * G9_STAGE;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = lb + j;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                *reinterpret_cast<u32x4 *>(base + b * G9_WB + r * 1024 + lane * 16) = stg[6 * j + r];
                *reinterpret_cast<u32x4 *>(base + G9_W + b * G9_XB + r * 1024 + lane * 16) = stg[6 * j + 3 + r];
            }
            *reinterpret_cast<uint32_t *>(base + G9_W + G9_X + b * 256 + lane * 4) = stg_dw[j];
        }
        *reinterpret_cast<uint32_t *>(base + G9_W + G9_X + G9_WD + lb * 128 + lane * 4) = stg_dx;
    };

    const int g = (wave >> 2) & 1, q = wave & 3;
    const int tt = 32 * (q & 1) + c;                       // this lane's token (A operand row) in the tile
    const int r0 = 64 * (q >> 1) + c, r1 = r0 + 32;        // this lane's weight rows (B operand columns)
    const int xo16 = h * 1024 + tt * 16, xo8 = 2048 + tt * 16 + 8 * (h ^ ((tt >> 4) & 1));
    const int sa = h ? G9_SCALE_1 : G9_SCALE_5;
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float acc0[16], acc1[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.0f;
    f32x16 S0 = fz, S1 = fz, P0 = fz, P1 = fz;
    u32x4 as = {0u, 0u, 0u, 0u}, bs0 = {0u, 0u, 0u, 0u}, bs1 = {0u, 0u, 0u, 0u};
    auto epi = [&](float *a, const f32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
        if constexpr (VAR & 2) {
            typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const f32x2 sv = {S[i], S[i + 1]}, pv = {P[i], P[i + 1]};
                f32x2 av = {a[i], a[i + 1]};
                av = __builtin_elementwise_fma(sv, pv, av);
                a[i] = av.x;
                a[i + 1] = av.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = fmaf(S[i], P[i], a[i]);
        }
    };
    struct Ops {
        i32x8 ax, bw0, bw1;
        uint32_t sx, sw0, sw1;
    };
    auto rd24 = [&](const uint8_t *p16, const uint8_t *p8) __attribute__((always_inline)) {
        const u32x4 u = *reinterpret_cast<const u32x4 *>(p16);
        const u32x2 v = *reinterpret_cast<const u32x2 *>(p8);
        const i32x8 r = {(int)u.x, (int)u.y, (int)u.z, (int)u.w, (int)v.x, (int)v.y, 0, 0};
        return r;
    };
    auto rd = [&](int st, int b) __attribute__((always_inline)) {
        const uint8_t *base = smem + (st % G9_NS) * G9_STAGE;
        const uint8_t *xb = base + G9_W + b * G9_XB, *wb = base + b * G9_WB;
        Ops o;
        o.ax = rd24(xb + xo16, xb + xo8);
        o.bw0 = rd24(wb + r0 * 16, wb + 2048 + r0 * 8);
        o.bw1 = rd24(wb + r1 * 16, wb + 2048 + r1 * 8);
        const uint16_t *wd = reinterpret_cast<const uint16_t *>(h ? zero : base + G9_W + G9_X + b * 256);
        o.sw0 = wd[h ? 0 : r0];
        o.sw1 = wd[h ? 0 : r1];
        o.sx = reinterpret_cast<const uint16_t *>(base + G9_W + G9_X + G9_WD + b * 128)[tt];
        return o;
    };
    // the rank-1 scale product d_x (x) d_w: one fp16 MFMA with only K element 0 nonzero (lanes 32-63
    // hold zeros in B), exact in f32.  VAR & 16: the K = 8 form v_mfma_f32_32x32x8_f16, 41 vs 51 nominal
    // cycles per instruction for the K = 16 form (tools/gemm_mb.hip VAR 42 / 43, four chains), same
    // output layout and the same products, so bitwise the same P
    auto scale_mfma = [&](const u32x4 &a, const u32x4 &b) __attribute__((always_inline)) {
        if constexpr (VAR & 16) {
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
            const u32x2 a2 = {a.x, a.y}, b2 = {b.x, b.y};
            return __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(half4, a2), __builtin_bit_cast(half4, b2), fz, 0, 0, 0);
        } else {
            return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), fz, 0, 0, 0);
        }
    };
    auto block = [&](const Ops &o) __attribute__((always_inline)) {
        as.x = o.sx;
        bs0.x = o.sw0;
        bs1.x = o.sw1;
        // the previous block's epilogues, then this block's four MFMAs back to back (gemm8's VAR 7 order)
        epi(acc0, S0, P0);
        epi(acc1, S1, P1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((VAR & 256) != 0) {
            // VAR 256: the two fp6 MFMAs, then the two fp16 ones (two format switches per burst, not four)
            S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw0, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
            S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw1, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
            P0 = scale_mfma(as, bs0);
            P1 = scale_mfma(as, bs1);
        } else {
            S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw0, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
            P0 = scale_mfma(as, bs0);
            S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw1, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
            P1 = scale_mfma(as, bs1);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync = [&]() __attribute__((always_inline)) {
        if (DIAG == 3) return;
        if constexpr (VAR & 8)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((G9_NS - 2) * G9_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    };

    const int nstages = (nb + G9_KB - 1) / G9_KB;
    if constexpr ((VAR & 128) != 0) {
        if (wave >= 8) __builtin_amdgcn_s_setprio(3);     // VAR 128: loader waves issue first
    }
    if constexpr (!(VAR & 8)) {
#pragma unroll
        for (int st = 0; st < G9_NS - 1; st++) issue(st);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((G9_NS - 2) * G9_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    }
    if constexpr (VAR & 8) {
        // separate code per role (the staging registers are not live in the compute loop), the same
        // barriers in each: one after the prologue, one per stage
        if (wave >= 8) {
            load_regs(0);
            store_regs(0);
            load_regs(1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            for (int s = 0; s < nstages; s++) {
                store_regs(s + 1);           // loaded during the previous stage (slot of stage s - 2: free)
                load_regs(s + 2);
                sync();
            }
        } else {
            __builtin_amdgcn_s_barrier();
            for (int s = 0; s < nstages; s++) {
                const int kb = s * G9_KB + 4 * g;
                if (DIAG != 1) {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (kb + j < nb) block(rd(s, 4 * g + j));
                }
                sync();
            }
        }
    } else
    for (int s = 0; s < nstages; s++) {
        issue(s + G9_NS - 1);
        const int kb = s * G9_KB + 4 * g;
        if (DIAG != 1 && wave < 8) {
            if constexpr (VAR & 4) {
                // nb even and kb even: blocks come in valid pairs
                if (kb < nb) {
                    Ops oa = rd(s, 4 * g), ob = rd(s, 4 * g + 1);
                    block(oa);
                    const bool more = kb + 2 < nb;
                    if (more) oa = rd(s, 4 * g + 2);
                    block(ob);
                    if (more) {
                        ob = rd(s, 4 * g + 3);
                        block(oa);
                        block(ob);
                    }
                }
            } else if constexpr (VAR & 32) {
                // per-stage VGPR bases, the block offsets as ds_read immediates: no address VALU per
                // block; the second weight tile's 8-byte part is read from its own (opaque) base, so
                // the compiler does not pair the two b64 reads into a ds_read2 + v_mov reassembly
                const uint32_t sb = (uint32_t)(s % G9_NS) * G9_STAGE;
                uint32_t xa = sb + G9_W + 4 * g * G9_XB + xo16, xb8 = sb + G9_W + 4 * g * G9_XB + xo8;
                uint32_t wa0 = sb + 4 * g * G9_WB + r0 * 16, wa1 = wa0 + 512;
                uint32_t w80 = sb + 4 * g * G9_WB + 2048 + r0 * 8, w81 = w80 + 256;
                uint32_t da = h ? (uint32_t)(G9_NS * G9_STAGE) : sb + G9_W + G9_X + 4 * g * 256 + r0 * 2;
                uint32_t xd = sb + G9_W + G9_X + G9_WD + 4 * g * 128 + tt * 2;
                asm volatile("" : "+v"(wa1), "+v"(w81));
                auto rdj = [&](int j) __attribute__((always_inline)) {
                    Ops o;
                    o.ax = rd24(smem + xa + j * G9_XB, smem + xb8 + j * G9_XB);
                    o.bw0 = rd24(smem + wa0 + j * G9_WB, smem + w80 + j * G9_WB);
                    o.bw1 = rd24(smem + wa1 + j * G9_WB, smem + w81 + j * G9_WB);
                    o.sw0 = *reinterpret_cast<const uint16_t *>(smem + da + j * 256);
                    o.sw1 = *reinterpret_cast<const uint16_t *>(smem + da + j * 256 + 64);
                    o.sx = *reinterpret_cast<const uint16_t *>(smem + xd + j * 128);
                    return o;
                };
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (kb + j >= nb) break;
                    block(rdj(j));
                }
            } else if constexpr (VAR & 1) {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (kb + j < nb) block(rd(s, 4 * g + j));
            } else {
                Ops o = rd(s, 4 * g);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (kb + j >= nb) break;
                    Ops nx = o;
                    if (j < 3) nx = rd(s, 4 * g + j + 1);
                    block(o);
                    o = nx;
                }
            }
        }
        sync();
    }
    epi(acc0, S0, P0);
    epi(acc1, S1, P1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float *red = reinterpret_cast<float *>(smem);
    if (wave >= 4 && wave < 8) {
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            *reinterpret_cast<float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4) = {acc0[i], acc0[i + 1], acc0[i + 2], acc0[i + 3]};
            *reinterpret_cast<float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4) = {acc1[i], acc1[i + 1], acc1[i + 2], acc1[i + 3]};
        }
    }
    __syncthreads();
    if (wave < 4) {
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            const float4 o0 = *reinterpret_cast<const float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4);
            const float4 o1 = *reinterpret_cast<const float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4);
            acc0[i] += o0.x; acc0[i + 1] += o0.y; acc0[i + 2] += o0.z; acc0[i + 3] += o0.w;
            acc1[i] += o1.x; acc1[i + 1] += o1.y; acc1[i + 2] += o1.z; acc1[i + 3] += o1.w;
        }
        const int row0 = m0 + r0, row1 = m0 + r1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int tk = n0 + 32 * (q & 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (tk < N) {
                if (row0 < M) y[(int64_t)tk * ldy + row0] = acc0[i];
                if (row1 < M) y[(int64_t)tk * ldy + row1] = acc1[i];
            }
        }
    }
}

int64_t gemm9_np(int64_t N) { return (N + 3) & ~(int64_t)3; }
size_t gemm9_x_bytes(int64_t K, int64_t N) { return (size_t)(K / QK) * gemm9_np(N) * 50; }
size_t gemm9_w_bytes(int64_t K, int64_t M) { return (size_t)((M + 127) / 128) * (K / QK) * 128 * 26; }

hipError_t gemm9_prep_x(const float *x, int64_t K, int64_t N, void *xws, hipStream_t s) {
    const int64_t nb = K / QK;
    if (N <= 0 || nb <= 0) return hipSuccess;
    if ((N + 7) / 8 > 65535) return hipErrorInvalidValue;
    const int64_t Np = gemm9_np(N);
    uint8_t *ximg = (uint8_t *)xws;
    uint16_t *xd16 = (uint16_t *)((char *)xws + (size_t)nb * Np * 48);
    (void)hipGetLastError();
    static const bool dpp = env_int("GGML_HIP_PREP9_DPP", 1) != 0;
    launch_k(dpp ? k_prep9_x<true> : k_prep9_x<false>, dim3((unsigned)((nb + 3) / 4), (unsigned)((N + 7) / 8)), dim3(256), 0, s, x, K, N, ximg, xd16, Np);
    return hipGetLastError();
}

hipError_t gemm9_prep_w(const void *W, int64_t K, int64_t M, void *wws, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t Mt = (M + 127) / 128;
    uint8_t *wimg = (uint8_t *)wws;
    uint16_t *wd16 = (uint16_t *)((char *)wws + (size_t)Mt * nb * G9_WB);
    (void)hipGetLastError();
    const int64_t items = Mt * (nb / 2);                  // (row tile, pair) items, 2 per 256-thread block
    launch_k(k_prep9_w, dim3((unsigned)((items + 1) / 2)), dim3(256), 0, s, (const uint8_t *)W, (int64_t)nb * Q4B, nb,
             (int)M, wimg, wd16);
    return hipGetLastError();
}

hipError_t gemm9_run(const void *wws, int64_t K, int64_t M, const void *xws, int64_t N, float *y, int64_t ldy,
                     hipStream_t s) {
    return gemm9_run_multi(1, &wws, &M, K, xws, N, &y, &ldy, s);
}

hipError_t gemm9_run_multi(int n, const void *const *wws, const int64_t *Mv, int64_t K, const void *xws, int64_t N,
                           float *const *yv, const int64_t *ldyv, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t Np = gemm9_np(N), Ny = (N + G9_BN - 1) / G9_BN;
    if (n < 1 || n > 4 || N <= 0 || nb <= 0) return hipErrorInvalidValue;
    G9Mats mats{};
    mats.n = n;
    mats.ny = (int)Ny;
    mats.tb[0] = 0;
    for (int i = 0; i < 4; i++) {
        const int k = i < n ? i : 0;
        const int64_t Mt = (Mv[k] + 127) / 128;
        mats.wimg[i] = (const uint8_t *)wws[k];
        mats.wd16[i] = (const uint16_t *)((const char *)wws[k] + (size_t)Mt * nb * G9_WB);
        mats.y[i] = yv[k];
        mats.ldy[i] = ldyv[k];
        mats.M[i] = (int)Mv[k];
        if (i < n) mats.tb[i + 1] = mats.tb[i] + (int)Mt;
    }
    for (int i = n; i < 4; i++) mats.tb[i + 1] = mats.tb[i];
    const int64_t tiles = (int64_t)mats.tb[n] * Ny;
    if (tiles >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    // GGML_HIP_GEMM9_XCD=0 restores the row-tile-fastest order (A/B)
    static const int xcd = env_int("GGML_HIP_GEMM9_XCD", 1);
    mats.xcd = xcd ? 1 : 0;
    const uint8_t *ximg = (const uint8_t *)xws;
    const uint16_t *xd16 = (const uint16_t *)((const char *)xws + (size_t)nb * Np * 48);
    if ((int64_t)nb * Np * 48 >= ((int64_t)1 << 31) || (int64_t)nb * G9_WB >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        for (auto k : {k_gemm9_q4_0<0, 0>, k_gemm9_q4_0<0, 1>, k_gemm9_q4_0<0, 4>, k_gemm9_q4_0<0, 9>, k_gemm9_q4_0<0, 17>,
                       k_gemm9_q4_0<0, 49>, k_gemm9_q4_0<0, 51>, k_gemm9_q4_0<0, 177>, k_gemm9_q4_0<0, 305>,
                       k_gemm9_q4_0<1, 49>, k_gemm9_q4_0<2, 49>, k_gemm9_q4_0<3, 49>, k_gemm9_q4_0<1, 9>,
                       k_gemm9_q4_0<4, 49>, k_gemm9_q4_0<5, 49>}) {
            hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, G9_LDS);
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
    static const int diag = env_int("GGML_HIP_GEMM_DIAG", 0);
    // GGML_HIP_GEMM9_VAR (A/B, tools/r3_g9var.sh, kernel medians, 2 interleaved rounds): 0 (prefetch one
    // block ahead through a copied operand set) 32.6-32.9 us at 4096x4096x512, 1 (no prefetch, default)
    // 25.9-26.0, 2 / 3 (packed epilogue) 38.5-38.7 / 26.7-26.8; k_gemm8 29.3-29.5 on the same boxes
    // 17 (= 1 with the scale product on the K = 8 fp16 MFMA, bitwise the same y; default since
    // tools/r3_g9p8.sh: kernel medians 26.44-26.52 vs 26.52-26.56 us at 4096^2 x 512, bench prefill
    // 0.370 / 0.377 vs 0.380 / 0.388 ms per layer in two rounds, VAR 17 run first in each)
    // 49 (= 17 with per-stage VGPR address bases, no address VALU per block; default since
    // tools/r3_g9p8.sh VA=17 VB=49: kernel medians 24.76-24.80 vs 26.76-26.84 us at 4096^2 x 512,
    // 4096 -> 11008 67.6-67.9 vs 72.2-74.1, 11008 -> 4096 55.8-57.7 vs 59.5-60.1)
    // 305 (= 49 with the burst ordered fp6, fp6, fp16, fp16; tools/r3_g9p8.sh VA=49 VB=305: 4096 -> 11008
    // 66.2-67.2 vs 68.1-68.5 us, 4096^2 25.0-25.1 vs 25.0-25.4, 11008 -> 4096 54.7-56.5 vs 55.4-56.5)
    static const int var = env_int("GGML_HIP_GEMM9_VAR", 305);
    auto kern = diag == 91 ? k_gemm9_q4_0<1, 49> : diag == 92 ? k_gemm9_q4_0<2, 49> : diag == 93 ? k_gemm9_q4_0<3, 49>
              : diag == 94 ? k_gemm9_q4_0<1, 9> : diag == 95 ? k_gemm9_q4_0<4, 49> : diag == 96 ? k_gemm9_q4_0<5, 49>
              : var == 0 ? k_gemm9_q4_0<0, 0> : var == 4 ? k_gemm9_q4_0<0, 4> : var == 9 ? k_gemm9_q4_0<0, 9>
              : var == 17 ? k_gemm9_q4_0<0, 17> : var == 49 ? k_gemm9_q4_0<0, 49>
              : var == 51 ? k_gemm9_q4_0<0, 51> : var == 177 ? k_gemm9_q4_0<0, 177>
              : var == 305 ? k_gemm9_q4_0<0, 305> : k_gemm9_q4_0<0, 1>;
    (void)hipGetLastError();
    launch_k(kern, dim3((unsigned)tiles), dim3(G9_THREADS), G9_LDS, s, mats, nb, ximg, xd16, Np, (int)N);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Split-K MFMA GEMM for small / medium token counts (9 <= N <= 128 by default).
//
// The LDS-staged GEMM above runs (M/64) x ceil(N/128) workgroups that each walk all of K, so for
// N <= 128 it uses a quarter of the chip and its time is one workgroup's K walk (~36 us at
// K = 4096).  Here a workgroup owns one 32-row x 32-token output tile and its SK waves split K into
// contiguous slices: each wave streams its slice's weight pairs (36 B per row) and q8_0 activations
// straight into registers through a DP-deep ring (no LDS staging, no barriers in the loop), runs
// the same per-block int8 MFMA + fp16 rank-1 scale MFMA + convert-free epilogue as the GEMM, and
// the SK partial tiles are summed through LDS in a fixed order (deterministic).  For N <= 32 every
// weight byte is read once.
template <int SK, int DP>
__global__ __launch_bounds__(SK * 64, 1) void k_gemm_sk_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes, int nb,
                                                              int M, const int8_t *__restrict__ xqs,
                                                              const float *__restrict__ xd, int N, int K,
                                                              float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) float red[];    // [SK][16][64] partial tiles
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
    // out-of-range rows / tokens read 0 through the descriptors (rows: d = 0 -> no contribution)
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W + (int64_t)m0 * rowbytes, (uint32_t)((int64_t)min(M - m0, 32) * rowbytes));
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(xqs + (int64_t)n0 * K, (uint32_t)((int64_t)min(N - n0, 32) * K));
    const __amdgpu_buffer_rsrc_t drs = make_rsrc(xd + (int64_t)n0 * nb, (uint32_t)((int64_t)min(N - n0, 32) * nb * 4));
    const int npairs = nb >> 1;
    const int ppw = (npairs + SK - 1) / SK;                         // pairs per wave
    const int p_begin = wave * ppw;
    const int p_end = min(npairs, p_begin + ppw);
    const int np = max(0, p_end - p_begin);

    struct Ring {
        u32x4 wa, wb;
        uint32_t wc;
        i32x4 x0, x1;
        float d0, d1;
    };
    auto issue = [&](int i) __attribute__((always_inline)) {        // pair p_begin + i (past the end: no traffic)
        Ring r;
        const bool v = i < np;
        const int p = p_begin + (v ? i : 0);
        const __amdgpu_buffer_rsrc_t w_ = v ? wrs : make_rsrc(W, 0);
        const __amdgpu_buffer_rsrc_t x_ = v ? xrs : make_rsrc(W, 0);
        const __amdgpu_buffer_rsrc_t d_ = v ? drs : make_rsrc(W, 0);
        const int woff = (int)(c * rowbytes) + 36 * p;
        r.wa = __builtin_amdgcn_raw_buffer_load_b128(w_, woff, 0, 0);
        r.wb = __builtin_amdgcn_raw_buffer_load_b128(w_, woff + 16, 0, 0);
        r.wc = __builtin_amdgcn_raw_buffer_load_b32(w_, woff + 32, 0, 0);
        const int xoff = c * K + 64 * p + 16 * h;
        r.x0 = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(x_, xoff, 0, 0));
        r.x1 = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(x_, xoff + 32, 0, 0));
        const u32x2 dd = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(d_, (c * nb + 2 * p) * 4, 0, 0));
        r.d0 = __uint_as_float(dd.x);
        r.d1 = __uint_as_float(dd.y);
        return r;
    };
    const int mg = 0x4B400000;
    const i32x16 im = {mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg};
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0.0f;
    auto block = [&](const i32x4 &xa, uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3, uint32_t dw16, float dx)
        __attribute__((always_inline)) {
        i32x4 wb;
        wb.x = (int)nib_to_i8x4(q0, 4 * h);
        wb.y = (int)nib_to_i8x4(q1, 4 * h);
        wb.z = (int)nib_to_i8x4(q2, 4 * h);
        wb.w = (int)nib_to_i8x4(q3, 4 * h);
        const i32x16 S = __builtin_amdgcn_mfma_i32_32x32x32_i8(xa, wb, im, 0, 0, 0);
        const u32x4 as = {h == 0 ? f2h(dx) : 0u, 0u, 0u, 0u};
        const u32x4 bs = {h == 0 ? dw16 : 0u, 0u, 0u, 0u};
        const f32x16 P = scale_rank1(as, bs);
#pragma unroll
        for (int i = 0; i < 16; i++) acc[i] = fmaf(__int_as_float(S[i]) - 12582912.0f, P[i], acc[i]);
    };
    auto process = [&](const Ring &r) __attribute__((always_inline)) {
        block(r.x0, __builtin_amdgcn_alignbyte(r.wa.y, r.wa.x, 2), __builtin_amdgcn_alignbyte(r.wa.z, r.wa.y, 2),
              __builtin_amdgcn_alignbyte(r.wa.w, r.wa.z, 2), __builtin_amdgcn_alignbyte(r.wb.x, r.wa.w, 2),
              r.wa.x & 0xFFFFu, r.d0);
        block(r.x1, r.wb.y, r.wb.z, r.wb.w, r.wc, r.wb.x >> 16, r.d1);
    };
    Ring ring[DP];
#pragma unroll
    for (int d = 0; d < DP; d++) ring[d] = issue(d);
    for (int i = 0; i < np; i += DP) {
#pragma unroll
        for (int d = 0; d < DP; d++) {
            if (i + d >= np) break;
            process(ring[d]);
            ring[d] = issue(i + d + DP);
        }
    }
    // fixed-order reduction of the SK partial tiles: red[w][i][lane]
#pragma unroll
    for (int i = 0; i < 16; i++) red[(wave * 16 + i) * 64 + lane] = acc[i];
    __syncthreads();
    for (int o = tid; o < 1024; o += SK * 64) {
        const int i = o >> 6, l = o & 63;
        float v = 0.0f;
        for (int w = 0; w < SK; w++) v += red[(w * 16 + i) * 64 + l];
        const int tok = n0 + 8 * (i >> 2) + 4 * (l >> 5) + (i & 3);
        const int row = m0 + (l & 31);
        if (tok < N && row < M) y[(int64_t)tok * ldy + row] = v;
    }
}

hipError_t gemm_sk_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N, float *y,
                        int64_t ldy, int num_cus, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    dim3 grid((unsigned)((M + 31) / 32), (unsigned)((N + 31) / 32));
    const int64_t tiles = (int64_t)grid.x * grid.y;
    static const int sk_env = env_int("GGML_HIP_GEMM_SK", 0);
    static const int dp = env_int("GGML_HIP_GEMM_SK_DP", 2);
    const int sk = sk_env ? sk_env : (tiles < 2 * (int64_t)num_cus ? 16 : 8);
    (void)hipGetLastError();  // report only this launch's error
    if (sk == 16 && dp == 4)
        launch_k((k_gemm_sk_q4_0<16, 4>), grid, dim3(1024), 16 * 16 * 64 * 4, s, (const uint8_t *)W, rowbytes,
                           nb, (int)M, xqs, xd, (int)N, (int)K, y, ldy);
    else if (sk == 8 && dp == 4)
        launch_k((k_gemm_sk_q4_0<8, 4>), grid, dim3(512), 8 * 16 * 64 * 4, s, (const uint8_t *)W, rowbytes,
                           nb, (int)M, xqs, xd, (int)N, (int)K, y, ldy);
    else if (sk == 16)
        launch_k((k_gemm_sk_q4_0<16, 2>), grid, dim3(1024), 16 * 16 * 64 * 4, s, (const uint8_t *)W, rowbytes,
                           nb, (int)M, xqs, xd, (int)N, (int)K, y, ldy);
    else
        launch_k((k_gemm_sk_q4_0<8, 2>), grid, dim3(512), 8 * 16 * 64 * 4, s, (const uint8_t *)W, rowbytes,
                           nb, (int)M, xqs, xd, (int)N, (int)K, y, ldy);
    return hipGetLastError();
}

hipError_t gemm_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                     float *y, int64_t ldy, hipStream_t s, const uint16_t *xd16) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    dim3 grid((unsigned)((M + GM_BM - 1) / GM_BM), (unsigned)((N + GM_BN - 1) / GM_BN));
    // GGML_HIP_GEMM_DIAG (diagnostic builds): 1 integer epilogue, 2 no MFMA, 3 no global loads,
    // 4 no LDS staging
    static const int diag = env_int("GGML_HIP_GEMM_DIAG", 0);
    static const int ver = env_int("GGML_HIP_GEMM_V", 7);
    if (ver == 7 && diag == 0) {
        static bool attr7 = false;
        if (!attr7) {
            hipError_t e = hipFuncSetAttribute((const void *)k_gemm7_q4_0, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               G7_LDS);
            if (e != hipSuccess) return e;
            attr7 = true;
        }
        (void)hipGetLastError();  // report only this launch's error
        if (!xd16) return hipErrorInvalidValue;
        launch_k(k_gemm7_q4_0, grid, dim3(GM_THREADS), G7_LDS, s, (const uint8_t *)W, rowbytes, nb, (int)M,
                           xqs, xd16, (int)N, (int)K, y, ldy);
        return hipGetLastError();
    }
    if (ver == 6) {
        // v6 diagnostics (GGML_HIP_GEMM_DIAG): 1 no epilogue VALU, 3 no global loads, 5 phase stamps,
        // 6/7 compute phase only (cvt / default epilogue).  GGML_HIP_GEMM_V=5: the previous kernel.
        auto k6 = diag == 1 ? k_gemm6_q4_0<1> : diag == 3 ? k_gemm6_q4_0<3> : diag == 5 ? k_gemm6_q4_0<5>
                : diag == 6 ? k_gemm6_q4_0<6> : diag == 7 ? k_gemm6_q4_0<7> : k_gemm6_q4_0<0>;
        static bool attr6 = false;
        if (!attr6) {
            for (auto k : {k_gemm6_q4_0<0>, k_gemm6_q4_0<1>, k_gemm6_q4_0<3>, k_gemm6_q4_0<5>, k_gemm6_q4_0<6>,
                           k_gemm6_q4_0<7>}) {
                hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   2 * G6_STAGE);
                if (e != hipSuccess) return e;
            }
            attr6 = true;
        }
        (void)hipGetLastError();  // report only this launch's error
        launch_k(k6, grid, dim3(GM_THREADS), 2 * G6_STAGE, s, (const uint8_t *)W, rowbytes, nb, (int)M,
                           xqs, xd, (int)N, (int)K, y, ldy);
        return hipGetLastError();
    }
    auto kern = diag == 1 ? k_gemm_q4_0<1> : diag == 2 ? k_gemm_q4_0<2> : diag == 3 ? k_gemm_q4_0<3>
              : diag == 4 ? k_gemm_q4_0<4> : diag == 5 ? k_gemm_q4_0<5> : k_gemm_q4_0<0>;
    static bool attr_set = false;       // up to 2 x 27 KB of dynamic LDS
    if (!attr_set) {
        for (auto k : {k_gemm_q4_0<0>, k_gemm_q4_0<1>, k_gemm_q4_0<2>, k_gemm_q4_0<3>, k_gemm_q4_0<4>,
                       k_gemm_q4_0<5>}) {
            hipError_t e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               2 * GM_STAGE);
            if (e != hipSuccess) return e;
        }
        attr_set = true;
    }
    (void)hipGetLastError();  // report only this launch's error
    launch_k(kern, grid, dim3(GM_THREADS), 2 * GM_STAGE, s, (const uint8_t *)W, rowbytes, nb,
                       (int)M, xqs, xd, (int)N, (int)K, y, ldy);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Exact mode (algo 4): every y bit-identical to the reference's x86 AVX2+FMA
// ggml_vec_dot_q4_0_q8_0 (ggml.c:2412-2435), which is a fixed fp32 schedule:
//   d      = fp32(d_w) * fp32(d_x)                         (exact: 11 x 11 significant bits)
//   lane j = sum of the 4 products of block elements 4j..4j+3 (bytes_from_nibbles_32 order:
//            elements 0..15 = low nibbles of qs[0..15], 16..31 = high nibbles), an exact int
//   acc_j  = fma(d, float(lane j), acc_j), block after block, for j = 0..7
//   y      = ((acc0+acc4) + (acc2+acc6)) + ((acc1+acc5) + (acc3+acc7))   (hsum_float_8, ggml.c:591)
// Eight threads per output row each run one lane's chain in block order, so all the freedom left
// is the memory schedule.  Chunks of EX_C = 64 blocks move global -> LDS by LDS-DMA only (no
// register staging, so nothing in flight is tied to a loop-carried register): an S-slot ring (2 at
// N = 1, 3 above), S - 1 chunks in flight, one counted `s_waitcnt vmcnt` + raw `s_barrier` per chunk (the slot refilled
// after the barrier is the one every wave finished before it).  Per slot:
//   weights: the 16 rows' 1152-byte row pieces as 16-byte units interleaved across rows (unit
//            (row r, piece k) at u = 16k + r, 9 x 1 KiB `buffer_load_dwordx4 ... lds` per wave):
//            the consumer's word D of row r sits at byte 256(D/4) + 16r + 4(D%4), bank
//            4r + D%4, so the 4 rows x 4 distinct words of a 32-lane group never conflict;
//   x:       int8 q8_0 bytes [col][block][32] (1 KiB per column-half, one DMA each);
//   d_x:     f32 [col][64] (one 256-byte dword DMA per column).
// Per step (block b of a chunk) lane j of row r: the qs word of elements 4j..4j+3 (an aligned
// word for odd blocks, v_alignbyte of two words for even ones), nib = 0..15 per byte, and lane
// j's exact integer sum_(4j..4j+3) (nib - 8) x = v_dot4_i32_i8(nib, x, v_dot4_i32_i8(x, -8)).
// The LDS operands of 8 steps are read one batch ahead.  The three hsum adds are xor-shuffles 4,
// 2, 1 within the row's 8 lanes (fp32 addition is commutative: lane k's acc_k + acc_{k^4} is the
// reference's r_k on both lanes).  x and d_x are the SoA quantizer's output (bit-exact bytes;
// d_x = the fp16-rounded scale as fp32), so d_w * d_x is the reference's d.
constexpr int EX_RB = 16;                            // output rows per workgroup (8 lanes each)
constexpr int EX_THREADS = EX_RB * 8;                // 128 = 2 waves
constexpr int EX_C = 64;                             // blocks per chunk (decode: EXC = 32, below)
// ring slots (S - 1 chunks in flight), per column count: decode (NC = 1) runs 2 slots = 41 KB of LDS,
// three workgroups per CU instead of two (tools/r2_exs.sh: exact decode 467 -> 532 tok/s; 4 slots 377);
// -DEX_SLOTS overrides every NC for A/B builds
#ifdef EX_SLOTS
constexpr int ex_slots(int) { return EX_SLOTS; }
#else
constexpr int ex_slots(int nc) { return nc == 1 ? 2 : 3; }
#endif

// EXC = blocks per chunk.  64: the weights of a chunk are 18 1-KiB DMAs, 9 per wave, and wave w loads
// half w of each x column.  32 (N = 1 only): 9 weight DMAs, 5 for wave 0 and 4 for wave 1, which loads
// the 1-KiB x column instead, so both waves still issue the same count (6 with the d_x DMA) and half
// the LDS per slot lets twice the workgroups share a CU (GGML_HIP_EXACT_C, tools/r3_exact_c.sh)
template <int NC, int EXC = EX_C, int SLOTS = 0>
struct ExLayout {
    static constexpr int WB = EX_RB * EXC * Q4B;                 // weight bytes per slot
    static constexpr int WI0 = (WB / 1024 + 1) / 2;              // weight DMAs of wave 0 / wave 1
    static constexpr int WI1 = WB / 1024 - WI0;
    static constexpr int XB = NC * EXC * 32;                     // x bytes per slot
    static constexpr int XW = EXC == 64 ? NC : (NC == 1 ? 1 : -1);   // x DMAs per wave (EXC 32: wave 1)
    static constexpr int DXW = (NC + 1) / 2;                     // d_x DMAs per wave per chunk
    static constexpr int DXB = DXW * 2 * 64 * 4;                 // d_x bytes per slot
    static constexpr int SLOT = WB + XB + DXB;
    static constexpr int OPS = EXC == 64 ? WI0 + NC + DXW : WI0 + DXW;   // vector-memory ops per wave per chunk
    static constexpr int S = SLOTS ? SLOTS : ex_slots(NC);       // ring slots
    static_assert(WB % 1024 == 0, "whole 1-KiB weight DMAs");
    static_assert(EXC == 64 ? WI0 == WI1 : (NC == 1 && WI0 == WI1 + 1), "equal DMA counts per wave");
    static_assert(OPS <= 63, "vmcnt immediate");
};

// Up to 4 matrices of the same K sharing x (siblings: wq|wk|wv, w1|w3) in one launch: workgroup
// rows [wg_begin[i], wg_begin[i+1]) of grid.x belong to matrix i (16 rows each, never straddling
// two matrices); the per-workgroup choice is written as sums of selected deltas (constant indices
// only: a dynamic index into the by-value struct becomes a scratch table)
struct ExMats {
    const uint8_t *W[4];
    float *y[4];
    int64_t ldy[4];
    int M[4];
    int wg_begin[5];
};

template <int NC, int EXC = EX_C, int SLOTS = 0>
__global__ __launch_bounds__(EX_THREADS) void k_mm_exact_q4_0(const ExMats mats, int64_t rowbytes,
                                                               int nb, const int8_t *__restrict__ xqs,
                                                               const float *__restrict__ xd, int N, int K) {
    using Lay = ExLayout<NC, EXC, SLOTS>;
    constexpr int EX_WB = Lay::WB;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int t = threadIdx.x, l64 = t & 63, lane = t & 7, r = t >> 3;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int q = lane & 3, shift = lane & 4;               // qs word q; low (j < 4) / high nibbles
    const int bx = blockIdx.x;
    const bool g1 = bx >= mats.wg_begin[1], g2 = bx >= mats.wg_begin[2], g3 = bx >= mats.wg_begin[3];
    const uint8_t *W = reinterpret_cast<const uint8_t *>(
        (uint64_t)mats.W[0] + (g1 ? (uint64_t)mats.W[1] - (uint64_t)mats.W[0] : 0) +
        (g2 ? (uint64_t)mats.W[2] - (uint64_t)mats.W[1] : 0) + (g3 ? (uint64_t)mats.W[3] - (uint64_t)mats.W[2] : 0));
    float *y = reinterpret_cast<float *>(
        (uint64_t)mats.y[0] + (g1 ? (uint64_t)mats.y[1] - (uint64_t)mats.y[0] : 0) +
        (g2 ? (uint64_t)mats.y[2] - (uint64_t)mats.y[1] : 0) + (g3 ? (uint64_t)mats.y[3] - (uint64_t)mats.y[2] : 0));
    const int64_t ldy = mats.ldy[0] + (g1 ? mats.ldy[1] - mats.ldy[0] : 0) + (g2 ? mats.ldy[2] - mats.ldy[1] : 0) +
                        (g3 ? mats.ldy[3] - mats.ldy[2] : 0);
    const int M = mats.M[0] + (g1 ? mats.M[1] - mats.M[0] : 0) + (g2 ? mats.M[2] - mats.M[1] : 0) +
                  (g3 ? mats.M[3] - mats.M[2] : 0);
    const int wb = (g1 ? mats.wg_begin[1] : 0) + (g2 ? mats.wg_begin[2] - mats.wg_begin[1] : 0) +
                   (g3 ? mats.wg_begin[3] - mats.wg_begin[2] : 0);
    const int m0 = (bx - wb) * EX_RB, n0 = blockIdx.y * NC;
    const int rows = min(EX_RB, M - m0), cols = min(NC, N - n0);
    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W + (int64_t)m0 * rowbytes, (uint32_t)((int64_t)rows * rowbytes));
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(xqs + (int64_t)n0 * K, (uint32_t)((int64_t)cols * K));
    const __amdgpu_buffer_rsrc_t drs = make_rsrc(xd + (int64_t)n0 * nb, (uint32_t)((int64_t)cols * nb * 4));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(W, 0);
    const int nchunks = (nb + EXC - 1) / EXC;
    // weight DMA i of this wave (slot instruction WI0*wave + i) covers units 64(WI0 wave + i) + l64:
    // row l64 & 15, piece 4(WI0 wave + i) + (l64 >> 4)
    const int wsrc = (l64 & 15) * (int)rowbytes + 16 * (4 * Lay::WI0 * wave + (l64 >> 4));

    auto issue = [&](int ch) __attribute__((always_inline)) {
        const bool valid = ch < nchunks;                    // past the end: counted, no traffic
        const int b0 = valid ? ch * EXC : 0;
        uint8_t *slot = smem + (ch % Lay::S) * Lay::SLOT;
        const __amdgpu_buffer_rsrc_t w_ = valid ? wrs : nul;
        const __amdgpu_buffer_rsrc_t x_ = valid ? xrs : nul;
        if (EXC == 64 || wave == 0) {
#pragma unroll
            for (int i = 0; i < Lay::WI0; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(w_, (lds_void_t *)(slot + 1024 * (Lay::WI0 * wave + i)), 16,
                                                         wsrc + b0 * Q4B + 64 * i, 0, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < Lay::WI1; i++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(w_, (lds_void_t *)(slot + 1024 * (Lay::WI0 * wave + i)), 16,
                                                         wsrc + b0 * Q4B + 64 * i, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(x_, (lds_void_t *)(slot + EX_WB), 16, b0 * 32 + 16 * l64, 0, 0, 0);
        }
        if constexpr (EXC == 64) {
#pragma unroll
            for (int c = 0; c < NC; c++)                     // wave w loads half w of each column
                __builtin_amdgcn_raw_ptr_buffer_load_lds(x_, (lds_void_t *)(slot + EX_WB + c * EXC * 32 + 1024 * wave), 16,
                                                         c * K + b0 * 32 + 1024 * wave + 16 * l64, 0, 0, 0);
        }
#pragma unroll
        for (int cc = 0; cc < Lay::DXW; cc++) {
            const int c = 2 * cc + wave;
            const __amdgpu_buffer_rsrc_t d_ = (valid && c < NC) ? drs : nul;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(d_, (lds_void_t *)(slot + EX_WB + Lay::XB + 256 * c), 4,
                                                     (c * nb + b0 + l64) * 4, 0, 0, 0);
        }
    };

    // per-lane byte offsets (within a slot) of word D = 9 p4 + q + delta of row r, p4 = pair % 4;
    // pair p = 4g + p4 adds 2304 g (= 36 g words) as an immediate
    auto woff = [&](int D) __attribute__((always_inline)) { return 256 * (D >> 2) + 16 * r + 4 * (D & 3); };
    int aE1[4], aE2[4], aO[4];
#pragma unroll
    for (int p4 = 0; p4 < 4; p4++) {
        aE1[p4] = woff(9 * p4 + q);
        aE2[p4] = woff(9 * p4 + q + 1);
        aO[p4] = woff(9 * p4 + 5 + q);
    }
    const int rbase = 16 * r;                               // + 256 (D>>2) + 4 (D&3) for lane-free D

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) acc[c] = 0.0f;

    // one step's operands
    struct Op {
        uint32_t wlo, whi, dwbits, x[NC];
        float dx[NC];
    };
    auto load_x = [&](Op &o, const uint8_t *slot, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            o.x[c] = reinterpret_cast<const uint32_t *>(slot + EX_WB + c * EXC * 32)[b * 8 + lane];
            o.dx[c] = reinterpret_cast<const float *>(slot + EX_WB + Lay::XB + 256 * c)[b];
        }
    };
    auto load_step = [&](Op &o, const uint8_t *slot, int b) __attribute__((always_inline)) {
        const int p = b >> 1, p4 = p & 3, g = p >> 2;
        const uint8_t *wsl = slot + 2304 * g;
        if (b & 1) {
            o.wlo = *reinterpret_cast<const uint32_t *>(wsl + aO[p4]);
            o.dwbits = *reinterpret_cast<const uint32_t *>(wsl + rbase + 256 * ((9 * p4 + 4) >> 2) + 4 * ((9 * p4 + 4) & 3));
        } else {
            o.wlo = *reinterpret_cast<const uint32_t *>(wsl + aE1[p4]);
            o.whi = *reinterpret_cast<const uint32_t *>(wsl + aE2[p4]);
            o.dwbits = *reinterpret_cast<const uint32_t *>(wsl + rbase + 256 * ((9 * p4) >> 2) + 4 * ((9 * p4) & 3));
        }
        load_x(o, slot, b);
    };
    auto use_step = [&](const Op &o, int b) __attribute__((always_inline)) {
        const uint32_t w = (b & 1) ? o.wlo : __builtin_amdgcn_alignbyte(o.whi, o.wlo, 2);
        const float dw = (b & 1) ? h2f(o.dwbits >> 16) : h2f(o.dwbits);
        const uint32_t nib = (w >> shift) & 0x0F0F0F0Fu;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int bias = __builtin_amdgcn_sdot4((int)o.x[c], (int)0xF8F8F8F8, 0, false);   // -8 sum x
            const int sgn = __builtin_amdgcn_sdot4((int)nib, (int)o.x[c], bias, false);
            acc[c] = __builtin_fmaf(dw * o.dx[c], (float)sgn, acc[c]);
        }
    };
    constexpr int BB = NC <= 2 ? 4 : 2;                      // steps per pipelined batch (lgkmcnt <= 15)

#pragma unroll
    for (int c = 0; c < Lay::S - 1; c++) issue(c);
    for (int ch = 0; ch < nchunks; ch++) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Lay::OPS * (Lay::S - 2)) : "memory");   // chunk ch landed
        __builtin_amdgcn_s_barrier();                       // everyone's landed; chunk ch-1 consumed
        issue(ch + Lay::S - 1);                             // into chunk ch-1's slot
        const uint8_t *slot = smem + (ch % Lay::S) * Lay::SLOT;
        const int cb = min(EXC, nb - ch * EXC);
        if (cb == EXC) {
            Op ops[2][BB];
#pragma unroll
            for (int b = 0; b < BB; b++) load_step(ops[0][b], slot, b);
#pragma unroll
            for (int i = 0; i < EXC / BB; i++) {
                // sched_barrier: keep the next batch's LDS reads ahead of this batch's math (the
                // scheduler otherwise pulls each read down to its use and waits on it)
                __builtin_amdgcn_sched_barrier(0);
                if (i + 1 < EXC / BB) {
#pragma unroll
                    for (int b = 0; b < BB; b++) load_step(ops[(i + 1) & 1][b], slot, (i + 1) * BB + b);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int b = 0; b < BB; b++) use_step(ops[i & 1][b], i * BB + b);
            }
            __builtin_amdgcn_sched_barrier(0);
        } else {
            for (int pp = 0; pp < cb / 2; pp++) {           // tail chunk (cb even), generic addressing
                Op o0, o1;
                const int p4 = pp & 3, g = pp >> 2;
                const uint8_t *wsl = slot + 2304 * g;
                o0.wlo = *reinterpret_cast<const uint32_t *>(wsl + woff(9 * p4 + q));
                o0.whi = *reinterpret_cast<const uint32_t *>(wsl + woff(9 * p4 + q + 1));
                o0.dwbits = *reinterpret_cast<const uint32_t *>(wsl + woff(9 * p4));
                o1.wlo = *reinterpret_cast<const uint32_t *>(wsl + woff(9 * p4 + 5 + q));
                o1.dwbits = *reinterpret_cast<const uint32_t *>(wsl + rbase + 256 * ((9 * p4 + 4) >> 2) +
                                                                4 * ((9 * p4 + 4) & 3));
                load_x(o0, slot, 2 * pp);
                load_x(o1, slot, 2 * pp + 1);
                use_step(o0, 0);
                use_step(o1, 1);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // no LDS-DMA may outlive the workgroup
#pragma unroll
    for (int c = 0; c < NC; c++) {
        float v = acc[c];
        v = v + __shfl_xor(v, 4, 8);       // r_k = acc_k + acc_{k+4}
        v = v + __shfl_xor(v, 2, 8);       // lane 0: r0 + r2, lane 1: r1 + r3
        v = v + __shfl_xor(v, 1, 8);       // lane 0: (r0 + r2) + (r1 + r3)
        if (lane == 0 && r < rows && c < cols) y[(int64_t)(n0 + c) * ldy + m0 + r] = v;
    }
}

template <int NC, int EXC = EX_C, int SLOTS = 0>
static hipError_t launch_exact(const ExMats &m, int n, int64_t K, const int8_t *xqs, const float *xd, int64_t N,
                               hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    const int lds = ExLayout<NC, EXC, SLOTS>::S * ExLayout<NC, EXC, SLOTS>::SLOT;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)k_mm_exact_q4_0<NC, EXC, SLOTS>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    dim3 grid((unsigned)m.wg_begin[n], (unsigned)((N + NC - 1) / NC));
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_mm_exact_q4_0<NC, EXC, SLOTS>, grid, dim3(EX_THREADS), lds, s, m, rowbytes, nb, xqs, xd, (int)N, (int)K);
    return hipGetLastError();
}

hipError_t mm_exact_q4_0_multi(int n, const void *const *W, const int64_t *M, int64_t K, const int8_t *xqs,
                               const float *xd, int64_t N, float *const *y, const int64_t *ldy, hipStream_t s) {
    if (n < 1 || n > 4) return hipErrorInvalidValue;
    ExMats m{};
    m.wg_begin[0] = 0;
    for (int i = 0; i < 4; i++) {
        const int j = i < n ? i : n - 1;                    // unused slots repeat the last matrix
        m.W[i] = (const uint8_t *)W[j];
        m.y[i] = y[j];
        m.ldy[i] = ldy[j];
        m.M[i] = (int)M[j];
        m.wg_begin[i + 1] = m.wg_begin[i] + (i < n ? (int)((M[i] + EX_RB - 1) / EX_RB) : 0);
    }
    static const int nc_env = env_int("GGML_HIP_EXACT_NC", 0);   // tuning: columns per workgroup
    // measured (tools/exact_nc.sh, 4096 x 4096): 8 columns best at N = 8, 2 at N = 40 and 512
    const int nc = nc_env ? nc_env : N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : 2;
    // decode chunk (GGML_HIP_EXACT_C 32 / 64 blocks) and its ring slots (GGML_HIP_EXACT_S, with 32: 2 / 3);
    // tools/r3_exact_c.sh, 2 interleaved rounds: 32 x 2 slots 549-551 tok/s, 64 x 2 530-533, 32 x 3 518-520
    static const int exc = env_int("GGML_HIP_EXACT_C", 32);
    static const int exs = env_int("GGML_HIP_EXACT_S", 2);
    if (nc == 1)
        return exc == 32 ? (exs == 3 ? launch_exact<1, 32, 3>(m, n, K, xqs, xd, N, s) : launch_exact<1, 32>(m, n, K, xqs, xd, N, s))
                         : launch_exact<1>(m, n, K, xqs, xd, N, s);
    if (nc == 2) return launch_exact<2>(m, n, K, xqs, xd, N, s);
    if (nc == 4) return launch_exact<4>(m, n, K, xqs, xd, N, s);
    return launch_exact<8>(m, n, K, xqs, xd, N, s);
}

hipError_t mm_exact_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                         float *y, int64_t ldy, hipStream_t s) {
    return mm_exact_q4_0_multi(1, &W, &M, K, xqs, xd, N, &y, &ldy, s);
}

// ---------------------------------------------------------------------------------------------
// multi-GPU gather compaction: slabs [nranks][N][max_rows] -> y[n][row_begin[r] + i]

__global__ __launch_bounds__(256) void k_scatter_slabs(const float *__restrict__ slabs, int nranks,
                                                         int64_t max_rows, const RowBegins row_begin,
                                                         int64_t N, float *__restrict__ y, int64_t ldy) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)nranks * N * max_rows;
    if (t >= total) return;
    const int64_t i = t % max_rows;
    const int64_t n = (t / max_rows) % N;
    const int r = (int)(t / (max_rows * N));
    const int64_t rb = row_begin.v[r], rows = row_begin.v[r + 1] - rb;
    if (i < rows) y[n * ldy + rb + i] = slabs[t];
}

hipError_t scatter_slabs(const float *slabs, int nranks, int64_t max_rows, const RowBegins &row_begin, int64_t N,
                         float *y, int64_t ldy, hipStream_t s) {
    const int64_t total = (int64_t)nranks * N * max_rows;
    if (total == 0) return hipSuccess;
    if (nranks > SCATTER_MAX_RANKS) return hipErrorInvalidValue;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_scatter_slabs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, slabs, nranks,
                       max_rows, row_begin, N, y, ldy);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// synthetic data: counter-based splitmix64 + Box-Muller (fp32)

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill_gaussian(float *__restrict__ dst, int64_t n, uint64_t seed, float mean,
                                                         float stdv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i >= n) return;
    const uint64_t z = splitmix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1)));
    const float u1 = ((float)(uint32_t)(z >> 40) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(uint32_t)(z & 0xFFFFFF) * (1.0f / 16777216.0f);        // [0, 1)
    const float r = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincosf(6.2831853071795864f * u2, &sn, &cs);
    dst[2 * i] = mean + stdv * r * cs;
    if (2 * i + 1 < n) dst[2 * i + 1] = mean + stdv * r * sn;
}

hipError_t fill_gaussian(float *dst, int64_t n, uint64_t seed, float mean, float stdv, hipStream_t s) {
    const int64_t pairs = (n + 1) / 2;
    if (pairs == 0) return hipSuccess;
    (void)hipGetLastError();  // report only this launch's error
    launch_k(k_fill_gaussian, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s, dst, n, seed, mean,
                       stdv);
    return hipGetLastError();
}

hipError_t gemm_read_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), sizeof(unsigned long long) * n, 0,
                               hipMemcpyDeviceToHost);
}

}  // namespace ghip
