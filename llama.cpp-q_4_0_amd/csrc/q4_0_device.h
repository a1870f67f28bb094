// q4_0_device.h — device helpers shared by the gfx950 (CDNA4) kernels of the ggml q4_0 x f32 mul_mat
// (internal to libggml_hip.so).  The kernels, one file per family:
//
// What each kernel restates (reference = ggml.c of Fcucgvhhhvjv/llama.cpp-q_4_0):
//   q4_0_quant.hip:
//   k_quantize_q8_0   quantize_row_q8_0, AVX2 branch ggml.c:1192-1275 (bit-exact: max|x|,
//                     d = amax/127.f (IEEE div), fp16(d) RNE, id = amax ? 127.f/amax : 0,
//                     q = sat8(round-half-even(x*id)))
//   k_quantize_q4_0   quantize_row_q4_0_reference ggml.c:918-953 (bit-exact)
//   k_dequantize_q4_0 dequantize_row_q4_0 ggml.c:1500-1518
//   q4_0_gemv.hip:
//   k_gemv_q4_0<NT>   mul_mat_q_f32 (ggml.c:11353-11411) for N <= 8 tokens: INIT (q8_0 of x)
//                     fused into the prologue (into LDS, once per workgroup), COMPUTE =
//                     ggml_vec_dot_q4_0_q8_0 (ggml.c:2339-2607) with one wave64 per weight row
//   q4_0_gemm.hip:
//   k_gemm7/8_q4_0    the same product for prefill batches on the int8 matrix cores
//                     (v_mfma_i32_32x32x32_i8: K=32 = exactly one q4_0/q8_0 block, so every
//                     MFMA yields the exact per-block integer sum the CPU computes); k_gemm7 reads
//                     the q4_0 bytes in place, k_gemm8 an int8 image of the weights
//   k_gemm9_q4_0      the default prefill GEMM on weight images: the same exact block sums from the
//                     block-scaled fp6 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 operands), as f32
//   q4_0_exact.hip:
//   k_mm_exact_q4_0   exact mode: the AVX2 branch's fp32 schedule, bit for bit
//
// Numerics: every per-block integer sum is exact (as on the CPU); the fp32 accumulation of
// d_w*d_x*sumi runs in a different order than AVX2's 8-lane fma chain, so y agrees with the
// reference within the fp32-accumulation bound (tests/parity.py), not bitwise.
#pragma once
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

// ggml's fp16 lookup tables table_silu_f16 / table_exp_f16 (ggml.c:4246-4254) hold the host libm's values
// rounded to fp16.  The backend builds them on the host (ggml-hip-ops.cpp) and checks once, on the device,
// the direct evaluation below against the table for every finite fp16 input (63,488 of each); when every
// one agrees bit for bit, the kernels get the table pointer tagged with bit 0 and evaluate instead of
// gathering (a table read is a 64-line random gather per wave instruction: the decode w2 GEMV's silu
// prologue was 4.9 us longer than without it).  Non-finite inputs always read the table.
__device__ __forceinline__ bool lut_direct(const uint16_t *t) { return ((uintptr_t)t & 1) != 0; }
__device__ __forceinline__ const uint16_t *lut_base(const uint16_t *t) {
    return reinterpret_cast<const uint16_t *>((uintptr_t)t & ~(uintptr_t)1);
}
__device__ __forceinline__ uint16_t silu_direct(uint32_t hb) {     // fp16(f / (1 + expf(-f))), f = fp16 hb
    const float f = h2f(hb);
    return (uint16_t)f2h(f / (1.0f + expf(-f)));
}
__device__ __forceinline__ uint16_t exp_direct(uint32_t hb) { return (uint16_t)f2h(expf(h2f(hb))); }
__device__ __forceinline__ uint16_t lut_silu(const uint16_t *t, uint32_t hb) {
    if (lut_direct(t) && (hb & 0x7C00u) != 0x7C00u) return silu_direct(hb);
    return lut_base(t)[hb & 0xFFFFu];
}
__device__ __forceinline__ uint16_t lut_exp(const uint16_t *t, uint32_t hb) {
    if (lut_direct(t) && (hb & 0x7C00u) != 0x7C00u) return exp_direct(hb);
    return lut_base(t)[hb & 0xFFFFu];
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
// e2m3_half as byte tables for v_perm_b32 (e2m3_codes4): four codes per dword, n = n0 .. n0 + 3
constexpr uint32_t e2m3_c(int n) {
    const uint32_t a = (uint32_t)(n < 0 ? -n : n), e = (uint32_t)(a >= 4u) + (uint32_t)(a >= 8u);
    return (n < 0 ? 0x20u : 0u) | ((a << (2u - e)) + 8u * e);
}
constexpr uint32_t e2m3_tab4(int n0) {
    return e2m3_c(n0) | (e2m3_c(n0 + 1) << 8) | (e2m3_c(n0 + 2) << 16) | (e2m3_c(n0 + 3) << 24);
}
// the e2m3_half codes of four 4-bit indices, one per byte: index i < 8 is n = i (the shared table),
// i >= 8 is looked up in (u0, u1) = the codes of the upper eight n (8..15 for q & 15, -8..-1 for q >> 4)
__device__ __forceinline__ uint32_t e2m3_codes4(uint32_t idx, uint32_t u0, uint32_t u1) {
    const uint32_t sel = idx & 0x07070707u;
    const uint32_t r0 = __builtin_amdgcn_perm(e2m3_tab4(4), e2m3_tab4(0), sel);
    const uint32_t r1 = __builtin_amdgcn_perm(u1, u0, sel);
    const uint32_t m = ((idx >> 3) & 0x01010101u) * 0xFFu;
    return (r1 & m) | (r0 & ~m);
}
// four 6-bit codes, one per byte -> the 24-bit field c0 | c1 << 6 | c2 << 12 | c3 << 18 (f6x4)
__device__ __forceinline__ uint32_t f6x4_bytes(uint32_t c) {
    return (c & 0x3Fu) | ((c >> 2) & 0xFC0u) | ((c >> 4) & 0x3F000u) | ((c >> 6) & 0xFC0000u);
}

// The k_gemm9 x image of one q8_0 block held by 8 consecutive lanes, 4 floats each (lane group
// sub = lane & 7; the q8_0 quantization of q8_block_lane): each lane's four q give four (q >> 4) and
// four (q & 15) codes (24 bits each; byte-table lookups, e2m3_codes4), and lanes 0-5 of the group
// assemble the block's six dwords of each half from their neighbours' fields.  Image layout (k_gemm9):
// codes [nb][3][Np][16 B] (part 0 = the first 16 B of the (q >> 4) codes, part 1 = those of the (q & 15)
// codes, part 2 = the last 8 B of both, swapped for tokens with bit 4 set) + fp16 d_x [nb][Np].  Every
// lane of the wave must call it (DPP); live = false: this lane's group stores nothing.  Offsets are
// 32-bit: the callers check nb * Np * 48 < 2^32 (x9_fits).  Shared by k_prep9_x and the producers that
// write the image beside their f32 output (ggml_ops.hip).
__device__ __forceinline__ void x9_store_lane(float4 v, int sub, int64_t n, int64_t b, bool live, uint8_t *ximg,
                                              uint16_t *xd16, int64_t Np) {
    uint32_t d16;
    int qsum;
    const uint32_t packed = q8_block_lane(v, d16, qsum);
    const uint32_t Fh = f6x4_bytes(e2m3_codes4(packed >> 4, e2m3_tab4(-8), e2m3_tab4(-4)));
    const uint32_t Fl = f6x4_bytes(e2m3_codes4(packed, e2m3_tab4(8), e2m3_tab4(12)));
    // dword k of a half: fields s and s + 1 shifted by off (k = 0..5 -> (s, off) = (0,0) (1,8) (2,16)
    // (4,0) (5,8) (6,16)); the fields of lanes +1 and +2 by DPP row shifts (groups of 8 lanes sit
    // inside 16-lane rows; lanes 6 and 7, which read past their group, store nothing): k < 3 takes
    // fields (own, +1), k >= 3 (+1, +2)
    const int k = sub < 6 ? sub : 5;
    const int off = 8 * (k % 3);
    const bool lo3 = k < 3;
    const uint32_t Fh1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Fh, 0x101, 0xF, 0xF, false);   // row_shl:1
    const uint32_t Fh2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Fh, 0x102, 0xF, 0xF, false);   // row_shl:2
    const uint32_t Fl1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Fl, 0x101, 0xF, 0xF, false);
    const uint32_t Fl2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)Fl, 0x102, 0xF, 0xF, false);
    const uint32_t h0 = lo3 ? Fh : Fh1, h1 = lo3 ? Fh1 : Fh2;
    const uint32_t l0 = lo3 ? Fl : Fl1, l1 = lo3 ? Fl1 : Fl2;
    if (!live || sub >= 6) return;
    const uint32_t dh = (h0 >> off) | (h1 << (24 - off)), dl = (l0 >> off) | (l1 << (24 - off));
    const uint32_t np = (uint32_t)Np, nn = (uint32_t)n, bb = (uint32_t)b;
    const int sw = (int)((nn >> 4) & 1u);
    uint32_t *p0 = reinterpret_cast<uint32_t *>(ximg + (bb * 3u * np + nn) * 16u);
    uint32_t *p1 = p0 + np * 4u;
    uint32_t *p2 = p1 + np * 4u;
    if (k < 4) {
        p0[k] = dh;
        p1[k] = dl;
    } else {
        p2[2 * sw + k - 4] = dh;
        p2[2 * (sw ^ 1) + k - 4] = dl;
    }
    if (sub == 0) xd16[bb * np + nn] = (uint16_t)d16;
}
// the image's offsets fit x9_store_lane's 32-bit arithmetic
static inline bool x9_fits(int64_t K, int64_t Np) { return K > 0 && Np > 0 && (K / 32) * Np * 48 < ((int64_t)1 << 32); }

// GGML_HIP_* tuning / test overrides read once (host)
static inline int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

}  // namespace ghip
