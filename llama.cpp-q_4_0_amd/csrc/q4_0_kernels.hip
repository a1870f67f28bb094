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
//                     MFMA yields the exact per-block integer sum the CPU computes)
//
// Numerics: every per-block integer sum is exact (as on the CPU); the fp32 accumulation of
// d_w*d_x*sumi runs in a different order than AVX2's 8-lane fma chain, so y agrees with the
// reference within the fp32-accumulation bound (tests/parity.py), not bitwise.
#include "q4_0_kernels.h"

#include <climits>
#include <cstdlib>

namespace ghip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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

// One q8_0 block spread over 8 consecutive lanes, 4 floats each (lane group g = lane>>3).
// Returns the packed int8x4 of this lane; d16 = fp16(amax/127.f); qsum = sum of the 32 q.
__device__ __forceinline__ uint32_t q8_block_lane(float4 v, uint32_t &d16, int &qsum) {
    float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    a = fmaxf(a, __shfl_xor(a, 1));
    a = fmaxf(a, __shfl_xor(a, 2));
    a = fmaxf(a, __shfl_xor(a, 4));
    const float d = a / 127.f;                         // correctly rounded (no fast-math)
    const float id = (a != 0.0f) ? 127.f / a : 0.0f;
    d16 = f2h(d);
    const int q0 = q8_round_sat(v.x * id), q1 = q8_round_sat(v.y * id);
    const int q2 = q8_round_sat(v.z * id), q3 = q8_round_sat(v.w * id);
    int s = q0 + q1 + q2 + q3;
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    qsum = s;
    return (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
           ((uint32_t)(q3 & 0xFF) << 24);
}

// ---------------------------------------------------------------------------------------------
// A5: q8_0 activation quantizer.  One lane per 4 floats, 8 lanes per block.

template <bool AOS>
__global__ __launch_bounds__(256) void k_quantize_q8_0(const float *__restrict__ x, int64_t K, int64_t total8,
                                                         uint8_t *__restrict__ aos, int8_t *__restrict__ qs,
                                                         float *__restrict__ dout) {
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
        if (sub == 0) dout[blk] = h2f(d16);
    }
}

hipError_t quantize_q8_0_aos(const float *x, int64_t K, int64_t N, void *xq8, hipStream_t s) {
    const int64_t total8 = N * (K / QK) * 8;
    if (total8 == 0) return hipSuccess;
    const int64_t grid = (total8 + 255) / 256;
    hipLaunchKernelGGL(k_quantize_q8_0<true>, dim3((unsigned)grid), dim3(256), 0, s, x, K, total8,
                       (uint8_t *)xq8, (int8_t *)nullptr, (float *)nullptr);
    return hipGetLastError();
}

hipError_t quantize_q8_0_soa(const float *x, int64_t K, int64_t N, int8_t *qs, float *d, hipStream_t s) {
    const int64_t total8 = N * (K / QK) * 8;
    if (total8 == 0) return hipSuccess;
    const int64_t grid = (total8 + 255) / 256;
    hipLaunchKernelGGL(k_quantize_q8_0<false>, dim3((unsigned)grid), dim3(256), 0, s, x, K, total8,
                       (uint8_t *)nullptr, qs, d);
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
            // separate rounding of v*id and +8.5 (no FMA contraction), as the C reference
            int q0 = (int)(signed char)(int)(__fmul_rn(v[j + t], id) + 8.5f);
            int q1 = (int)(signed char)(int)(__fmul_rn(v[j + t + QK / 2], id) + 8.5f);
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
    hipLaunchKernelGGL(k_quantize_q4_0, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, s, w, nblocks,
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
    hipLaunchKernelGGL(k_dequantize_q4_0, dim3((unsigned)((nblocks * 16 + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t *)wq, nblocks, w);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// GEMV (decode, N <= 8).
//
// Lane p of a wave owns block pair p of a 64-pair chunk of one weight row.  A pair is 36 bytes
// (9 dwords): the 18-byte blocks of a row start 4-byte aligned every second block, so a pair
// is always dword aligned and the 64 lanes of one load read 2,304 contiguous bytes (a whole
// K=4096 row).  Loads are buffer_load_dwordx4/x4/x1 through the row's descriptor
// (out-of-row lanes read 0, no fault).  The even block's qs are re-aligned with
// v_alignbyte_b32.  x is quantized once per workgroup into LDS (q8_0 ints + fp32 d +
// 8*sum(q)); the q4_0 nibbles enter v_dot4c_i32_i8 unsigned (0..15) and the -8 offset is
// applied once per block as -8*sum(q):  sum((n-8)*q) = sum(n*q) - 8*sum(q).
//
// Schedule: the activation loads are issued first, then the wave's first weight chunk, so
// the q8_0 prologue overlaps the first HBM round trip; after the prologue each wave walks its
// (row, chunk) items with the next chunk's loads in flight while the current one computes.

static constexpr int GEMV_THREADS = 1024;
static constexpr int GEMV_LDS_MAX = 64 * 1024;
static constexpr int GEMV_PRO = 4;          // activation float4 loads in flight per thread

__device__ __forceinline__ int dot_q4_q8(uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3,
                                         const uint32_t *__restrict__ xb) {
    const u32x4 xl = *reinterpret_cast<const u32x4 *>(xb);      // elems 0..15
    const u32x4 xh = *reinterpret_cast<const u32x4 *>(xb + 4);  // elems 16..31
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

template <int NT>
__global__ __launch_bounds__(GEMV_THREADS) void k_gemv_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes,
                                                             int nb, int M, const float *__restrict__ x, int K,
                                                             float *__restrict__ y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t *xq = lds;                                             // [NT][nb][8] int8x4
    float *xd = reinterpret_cast<float *>(lds + NT * nb * 8);      // [NT][nb]
    int *xs = reinterpret_cast<int *>(xd + NT * nb);               // [NT][nb] 8*sum(q)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwaves = GEMV_THREADS / 64;
    const int npairs = nb >> 1;
    const int nchunk = (npairs + 63) >> 6;
    const int rstride = gridDim.x * nwaves;
    const int row0 = blockIdx.x * nwaves + wave;
    const int nrows_w = row0 < M ? (M - 1 - row0) / rstride + 1 : 0;
    const int nitems = nrows_w * nchunk;                            // (row, chunk) items of this wave

    // ---- INIT: q8_0 of the NT activation rows into LDS, first weight chunk issued in between.
    // x of the NT tokens is contiguous ([NT][K] f32), so thread t's float4 is at byte 16*t.  All
    // loads are unconditional buffer loads (out-of-range -> 0, no traffic) so the compiler can
    // count vmcnt exactly: the q8_0 math waits for the activations only, not the weights.
    const int total = NT * nb * 8;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, (uint32_t)total * 16u);
    auto quantize_into_lds = [&](const u32x4 &raw, int t) {
        if (t < total) {                                            // whole 8-lane groups agree
            const float4 v = make_float4(__uint_as_float(raw.x), __uint_as_float(raw.y),
                                         __uint_as_float(raw.z), __uint_as_float(raw.w));
            uint32_t d16;
            int qsum;
            const uint32_t packed = q8_block_lane(v, d16, qsum);
            xq[t] = packed;
            if ((t & 7) == 0) {
                xd[t >> 3] = h2f(d16);
                xs[t >> 3] = 8 * qsum;
            }
        }
    };
    u32x4 xv[GEMV_PRO];
#pragma unroll
    for (int i = 0; i < GEMV_PRO; i++)
        xv[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (tid + i * GEMV_THREADS), 0, 0);
    PairRegs cur = load_pair(W + (int64_t)(nitems > 0 ? row0 : 0) * rowbytes, nitems > 0 ? rowbytes : 0, lane);
#pragma unroll
    for (int i = 0; i < GEMV_PRO; i++) quantize_into_lds(xv[i], tid + i * GEMV_THREADS);
    for (int base = GEMV_PRO * GEMV_THREADS; base < total; base += GEMV_PRO * GEMV_THREADS) {
#pragma unroll
        for (int i = 0; i < GEMV_PRO; i++)
            xv[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * GEMV_THREADS), 0, 0);
#pragma unroll
        for (int i = 0; i < GEMV_PRO; i++) quantize_into_lds(xv[i], base + tid + i * GEMV_THREADS);
    }
    __syncthreads();

    // ---- COMPUTE: stream the wave's (row, chunk) items with one item in flight.  Two named
    // register sets (no register copies: a copy would force a wait on the in-flight loads).
    float acc[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) acc[n] = 0.0f;
    auto item_row = [&](int it) { return row0 + (it / nchunk) * rstride; };
    auto issue = [&](int it) {
        const bool valid = it < nitems;                             // past the end: zero-size descriptor
        const int r = valid ? item_row(it) : row0;
        return load_pair(W + (int64_t)r * rowbytes, valid ? rowbytes : 0, 64 * (it % nchunk) + lane);
    };
    auto process = [&](const PairRegs &v, int it) {
        const int chunk = it % nchunk;
        const int p = 64 * chunk + lane;
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
                const float2 dx = *reinterpret_cast<const float2 *>(xd + bA);
                const int2 sx = *reinterpret_cast<const int2 *>(xs + bA);
                const int sA = dot_q4_q8(qA0, qA1, qA2, qA3, xq + bA * 8) - sx.x;
                const int sB = dot_q4_q8(v.b.y, v.b.z, v.b.w, v.c, xq + bA * 8 + 8) - sx.y;
                acc[n] = fmaf((float)sA, dA * dx.x, acc[n]);
                acc[n] = fmaf((float)sB, dB * dx.y, acc[n]);
            }
        }
        if (chunk == nchunk - 1) {                                  // row complete: reduce + store
            float out = 0.0f;
#pragma unroll
            for (int n = 0; n < NT; n++) {
                float t = acc[n];
                t += __shfl_xor(t, 32);
                t += __shfl_xor(t, 16);
                t += __shfl_xor(t, 8);
                t += __shfl_xor(t, 4);
                t += __shfl_xor(t, 2);
                t += __shfl_xor(t, 1);
                out = (lane == n) ? t : out;
                acc[n] = 0.0f;
            }
            if (lane < NT) y[(int64_t)lane * ldy + item_row(it)] = out;
        }
    };
    PairRegs nxt;
    for (int it = 0; it < nitems; it += 2) {
        nxt = issue(it + 1);
        process(cur, it);
        if (it + 1 >= nitems) break;
        cur = issue(it + 2);
        process(nxt, it + 1);
    }
}

int gemv_max_tokens(int64_t K) {
    const int64_t nb = K / QK;
    int nt = 8;
    while (nt > 0 && nt * nb * 40 > GEMV_LDS_MAX) nt--;
    return nt;
}

static int g_gemv_wg_per_cu = 0;

template <int NT>
static hipError_t launch_gemv(const void *W, int64_t K, int64_t M, const float *x, float *y, int64_t ldy,
                              const DeviceInfo &dev, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    const size_t lds = (size_t)NT * nb * 40;
    if (g_gemv_wg_per_cu == 0) {
        const char *e = getenv("GGML_HIP_GEMV_WG_PER_CU");
        g_gemv_wg_per_cu = e ? atoi(e) : 2;
        if (g_gemv_wg_per_cu < 1) g_gemv_wg_per_cu = 1;
    }
    const int64_t need = (M + GEMV_THREADS / 64 - 1) / (GEMV_THREADS / 64);
    const int64_t cap = (int64_t)dev.num_cus * g_gemv_wg_per_cu;
    const unsigned grid = (unsigned)(need < cap ? need : cap);
    hipLaunchKernelGGL(k_gemv_q4_0<NT>, dim3(grid), dim3(GEMV_THREADS), lds, s, (const uint8_t *)W, rowbytes, nb,
                       (int)M, x, (int)K, y, ldy);
    return hipGetLastError();
}

hipError_t gemv_q4_0(const void *W, int64_t K, int64_t M, const float *x, int64_t N, float *y, int64_t ldy,
                     const DeviceInfo &dev, hipStream_t s) {
    switch (N) {
        case 1: return launch_gemv<1>(W, K, M, x, y, ldy, dev, s);
        case 2: return launch_gemv<2>(W, K, M, x, y, ldy, dev, s);
        case 3: return launch_gemv<3>(W, K, M, x, y, ldy, dev, s);
        case 4: return launch_gemv<4>(W, K, M, x, y, ldy, dev, s);
        case 5: return launch_gemv<5>(W, K, M, x, y, ldy, dev, s);
        case 6: return launch_gemv<6>(W, K, M, x, y, ldy, dev, s);
        case 7: return launch_gemv<7>(W, K, M, x, y, ldy, dev, s);
        case 8: return launch_gemv<8>(W, K, M, x, y, ldy, dev, s);
        default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------------------------
// GEMM (prefill): workgroup tile = 128 weight rows x 64 tokens, 4 waves as 2 (rows) x 2 (tokens);
// each wave owns two 32x32 MFMA tiles (64 rows x 32 tokens).  K advances 4 blocks per stage.
//
// MFMA roles: A = activations (token = MFMA row), B = weights (weight row = MFMA column), so
// D[token][wrow] has the weight row on the lane and the output store y[token][m0 + lane] is a
// contiguous 128-byte segment per register.  Lane (c, h) = (lane&31, lane>>5) supplies k-half h
// of its row/column: activations bytes 16h..16h+15 of the q8_0 block, weights the low (h=0) or
// high (h=1) nibbles of the 16 qs bytes = elements 16h..16h+15.  The i32 result of one MFMA is
// the exact block sum; the epilogue applies d_x[token]*d_w[row] in fp32.

static constexpr int GM_BM = 128, GM_BN = 64, GM_KB = 4;
static constexpr int GM_WSTR = GM_KB * Q4B + 4;     // 76 B: 19 dwords (odd) -> conflict-free b32 reads
static constexpr int GM_XSTR = GM_KB * QK + 16;     // 144 B: conflict-free ds_read_b128 per 16-lane group
static constexpr int GM_WDW = GM_KB * Q4B / 4;      // 18 dwords of raw weights per row per stage

__device__ __forceinline__ uint32_t nib_to_i8x4(uint32_t q, int shift) {
    const uint32_t n = (q >> shift) & 0x0F0F0F0Fu;                 // 0..15 per byte
    return ((n | 0x80808080u) - 0x08080808u) ^ 0x80808080u;      // n - 8 as int8, no cross-byte borrow
}

__global__ __launch_bounds__(256) void k_gemm_q4_0(const uint8_t *__restrict__ W, int64_t rowbytes, int nb, int M,
                                                   const int8_t *__restrict__ xqs, const float *__restrict__ xd,
                                                   int N, int K, float *__restrict__ y, int64_t ldy) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[GM_BM * GM_WSTR + GM_BN * GM_XSTR + GM_KB * GM_BN * 4];
    uint8_t *wl = smem;                                    // [BM][WSTR] raw block_q4_0 bytes
    uint8_t *xl = smem + GM_BM * GM_WSTR;                  // [BN][XSTR] int8 activations
    float *dl = reinterpret_cast<float *>(xl + GM_BN * GM_XSTR);   // [KB][BN] d_x

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave & 1, wt = wave >> 1;
    const int c = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.x * GM_BM;
    const int n0 = blockIdx.y * GM_BN;

    // whole-operand descriptors: out-of-range rows / tokens read as 0
    const int64_t wbytes = (int64_t)M * rowbytes;
    const __amdgpu_buffer_rsrc_t wr_rsrc = make_rsrc(W + (int64_t)m0 * rowbytes,
                                                     (uint32_t)(wbytes - (int64_t)m0 * rowbytes));
    const __amdgpu_buffer_rsrc_t xr_rsrc = make_rsrc(xqs + (int64_t)n0 * K,
                                                     (uint32_t)((int64_t)(N - n0) * K));

    // staging registers (prefetch of stage s+1 while stage s computes)
    uint32_t wreg[9];
    u32x4 xreg[2];
    float dreg;

    auto load_stage = [&](int kb0) {
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const int idx = tid + 256 * i;                 // 0 .. 128*18-1
            const int r = idx / GM_WDW, dw = idx - r * GM_WDW;
            wreg[i] = __builtin_amdgcn_raw_buffer_load_b32(wr_rsrc, (int)(r * rowbytes + kb0 * Q4B + 4 * dw), 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + 256 * i;                 // 0 .. 64*8-1
            const int t = idx >> 3, part = idx & 7;
            xreg[i] = __builtin_amdgcn_raw_buffer_load_b128(xr_rsrc, t * K + kb0 * QK + 16 * part, 0, 0);
        }
        {
            const int b = tid >> 6, t = tid & 63;          // KB*BN == 256
            dreg = (n0 + t < N && kb0 + b < nb) ? xd[(int64_t)(n0 + t) * nb + kb0 + b] : 0.0f;
        }
    };
    auto store_stage = [&]() {
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const int idx = tid + 256 * i;
            const int r = idx / GM_WDW, dw = idx - r * GM_WDW;
            *reinterpret_cast<uint32_t *>(wl + r * GM_WSTR + 4 * dw) = wreg[i];
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + 256 * i;
            const int t = idx >> 3, part = idx & 7;
            *reinterpret_cast<u32x4 *>(xl + t * GM_XSTR + 16 * part) = xreg[i];
        }
        dl[tid] = dreg;
    };

    float acc[2][16];
#pragma unroll
    for (int ct = 0; ct < 2; ct++)
#pragma unroll
        for (int i = 0; i < 16; i++) acc[ct][i] = 0.0f;

    load_stage(0);
    for (int kb0 = 0; kb0 < nb; kb0 += GM_KB) {
        __syncthreads();                                   // previous stage's LDS reads done
        store_stage();
        __syncthreads();
        if (kb0 + GM_KB < nb) load_stage(kb0 + GM_KB);     // in flight during this stage's MFMAs
#pragma unroll
        for (int b = 0; b < GM_KB; b++) {
            if (kb0 + b >= nb) break;
            const int tok = 32 * wt + c;
            const u32x4 af = *reinterpret_cast<const u32x4 *>(xl + tok * GM_XSTR + 32 * b + 16 * h);
            // d_x of the 16 tokens this lane's accumulator registers hold: 8q + 4h + {0..3}
            float dx[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 f = *reinterpret_cast<const float4 *>(dl + b * GM_BN + 32 * wt + 8 * q + 4 * h);
                dx[4 * q] = f.x; dx[4 * q + 1] = f.y; dx[4 * q + 2] = f.z; dx[4 * q + 3] = f.w;
            }
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const int wrow = 64 * wr + 32 * ct + c;
                const uint32_t *wp = reinterpret_cast<const uint32_t *>(wl + wrow * GM_WSTR);
                uint32_t q0, q1, q2, q3, dbits;
                if ((b & 1) == 0) {                        // block starts dword aligned: d | qs0 qs1
                    const int o = (9 * b) / 2;
                    const uint32_t d0 = wp[o], d1 = wp[o + 1], d2 = wp[o + 2], d3 = wp[o + 3], d4 = wp[o + 4];
                    dbits = d0 & 0xFFFFu;
                    q0 = __builtin_amdgcn_alignbyte(d1, d0, 2);
                    q1 = __builtin_amdgcn_alignbyte(d2, d1, 2);
                    q2 = __builtin_amdgcn_alignbyte(d3, d2, 2);
                    q3 = __builtin_amdgcn_alignbyte(d4, d3, 2);
                } else {                                   // d in the upper half of the previous dword
                    const int o = (9 * b + 1) / 2;
                    dbits = wp[o - 1] >> 16;
                    q0 = wp[o]; q1 = wp[o + 1]; q2 = wp[o + 2]; q3 = wp[o + 3];
                }
                const int sh = 4 * h;
                i32x4 bf;
                bf.x = (int)nib_to_i8x4(q0, sh);
                bf.y = (int)nib_to_i8x4(q1, sh);
                bf.z = (int)nib_to_i8x4(q2, sh);
                bf.w = (int)nib_to_i8x4(q3, sh);
                i32x16 cz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
                const i32x16 cv = __builtin_amdgcn_mfma_i32_32x32x32_i8((i32x4)af, bf, cz, 0, 0, 0);
                const float dw = h2f(dbits);
#pragma unroll
                for (int i = 0; i < 16; i++) acc[ct][i] = fmaf((float)cv[i], dw * dx[i], acc[ct][i]);
            }
        }
    }

    // epilogue: acc[ct][i] = y[token(i)][row]; token(i) = 32wt + (i&3) + 8(i>>2) + 4h
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const int row = m0 + 64 * wr + 32 * ct + c;
        if (row >= M) continue;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int tok = n0 + 32 * wt + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (tok < N) y[(int64_t)tok * ldy + row] = acc[ct][i];
        }
    }
}

hipError_t gemm_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                     float *y, int64_t ldy, hipStream_t s) {
    const int nb = (int)(K / QK);
    const int64_t rowbytes = (int64_t)nb * Q4B;
    dim3 grid((unsigned)((M + GM_BM - 1) / GM_BM), (unsigned)((N + GM_BN - 1) / GM_BN));
    hipLaunchKernelGGL(k_gemm_q4_0, grid, dim3(256), 0, s, (const uint8_t *)W, rowbytes, nb, (int)M, xqs, xd,
                       (int)N, (int)K, y, ldy);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// multi-GPU gather compaction: slabs [nranks][N][max_rows] -> y[n][row_begin[r] + i]

__global__ __launch_bounds__(256) void k_scatter_slabs(const float *__restrict__ slabs, int nranks,
                                                         int64_t max_rows, const int64_t *__restrict__ row_begin,
                                                         int64_t N, float *__restrict__ y, int64_t ldy) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)nranks * N * max_rows;
    if (t >= total) return;
    const int64_t i = t % max_rows;
    const int64_t n = (t / max_rows) % N;
    const int r = (int)(t / (max_rows * N));
    const int64_t rows = row_begin[r + 1] - row_begin[r];
    if (i < rows) y[n * ldy + row_begin[r] + i] = slabs[t];
}

hipError_t scatter_slabs(const float *slabs, int nranks, int64_t max_rows, const int64_t *row_begin_dev, int64_t N,
                         float *y, int64_t ldy, hipStream_t s) {
    const int64_t total = (int64_t)nranks * N * max_rows;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_slabs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, slabs, nranks,
                       max_rows, row_begin_dev, N, y, ldy);
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
    hipLaunchKernelGGL(k_fill_gaussian, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s, dst, n, seed, mean,
                       stdv);
    return hipGetLastError();
}

}  // namespace ghip
