// q4_0_quant.hip — the bit-exact q8_0 / q4_0 quantizers and q4_0 dequantizer (A5, A3, A4), the multi-GPU gather
// compaction and the bench's synthetic-input generator.
// Shared device helpers and the HBM layouts: q4_0_device.h / q4_0_kernels.h.
#include "q4_0_device.h"

namespace ghip {

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

}  // namespace ghip
