// Compute-phase microbenchmark for the prefill GEMM (round 3): the per-block work of the q4_0 x q8_0
// int8-MFMA GEMM with its operands already in LDS (no global loads, no barriers), to find the loop
// structure that runs closest to the MFMA/VALU issue floor before building the full kernel.
//
// Per 32x32 output tile and q4_0 block: one v_mfma_i32_32x32x32_i8 (exact integer block sum), the
// rank-1 scale d_x (x) d_w (one f16 MFMA, or 16 VALU multiplies), and the epilogue acc += (S - bias)*P.
// Variants (template VAR):
//   0  gemm7's structure: 1 tile per wave, (S, P) double-buffered, operands read one block ahead
//   1  2 token tiles per wave sharing the weight operand: mfma(t0,b) epi(t1,b-1) mfma(t1,b) epi(t0,b)
//   2  VAR 1 with sched_group_barrier interleaving (1 MFMA : 8 VALU)
//   3  VAR 0 with the scale product by VALU (16 v_mul_f32 from fp32 d_x read 4 at a time)
//   4  4 tiles per wave (2 row x 2 token), 1 MFMA chain set per tile
//   (... 5-35: see the variant comments)
//   36 VAR21 with the block sum from the block-scaled fp6 MFMA (f32 result: no conversion), 37 its MFMAs
//      alone; 38 / 39 four independent chains of fp6 / i8 MFMAs only (issue rate of each instruction)
// Usage: gemm_mb [nblk]; prints us per launch and cycles per (tile x block) per SIMD at 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int R = 4;              // LDS ring of blocks
constexpr int BN = 128, BM = 64;  // workgroup tile (tokens x rows)
constexpr int LA = R * BN * 32;   // int8 x
constexpr int LB = R * BM * 32;   // int8 w
constexpr int LSX = R * BN * 4;   // fp32/fp16 d_x
constexpr int LSW = R * BM * 4;   // d_w
constexpr int LDS = LA + LB + LSX + LSW + 512;

__device__ __forceinline__ int hoff(int r, int half) { return r * 32 + 16 * (half ^ ((r >> 3) & 1)); }

template <int VAR>
__global__ __launch_bounds__(512, 2) void k_mb(const uint8_t *src, float *out, int nblk) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid * 4; i < LDS - 512; i += 512 * 4) *(uint32_t *)(lds + i) = *(const uint32_t *)(src + i);
    uint16_t *sx16 = (uint16_t *)(lds + LA + LB);
    uint16_t *sw16 = (uint16_t *)(lds + LA + LB + LSX);
    const float *sx32 = (const float *)(lds + LA + LB);
    uint16_t *zero = (uint16_t *)(lds + LDS - 512);
    if (tid < 128) ((uint32_t *)zero)[tid] = 0;
    // small finite fp16 scales (so P stays finite): overwrite with 1/1024-ish values
    for (int i = tid; i < R * BN; i += 512) sx16[i] = 0x1400 + (i & 255);
    for (int i = tid; i < R * BM; i += 512) sw16[i] = 0x1400 + (i & 127);
    __syncthreads();
    const int c = lane & 31, h = lane >> 5;
    const int mg = 0x4B400000;
    const i32x16 im = {mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg, mg};
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float acc[4][16];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int i = 0; i < 16; i++) acc[t][i] = 0.f;

    auto epi = [&](float *a, const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; i++) a[i] = fmaf(__int_as_float(S[i]) - 12582912.0f, P[i], a[i]);
    };
    auto rdA = [&](int b, int tok) __attribute__((always_inline)) {
        return *(const i32x4 *)(lds + (b & (R - 1)) * BN * 32 + hoff(tok, h));
    };
    auto rdB = [&](int b, int row) __attribute__((always_inline)) {
        return *(const i32x4 *)(lds + LA + (b & (R - 1)) * BM * 32 + hoff(row, h));
    };
    auto rdSX = [&](int b, int tok) __attribute__((always_inline)) { return (uint32_t)sx16[(b & (R - 1)) * BN + tok]; };
    auto rdSW = [&](int b, int row) __attribute__((always_inline)) {
        return (uint32_t)(h ? zero : sw16)[(b & (R - 1)) * BM + row];
    };
    auto mfma2 = [&](i32x4 a, i32x4 bb, uint32_t sx, uint32_t sw, i32x16 &S, f32x16 &P) __attribute__((always_inline)) {
        S = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bb, im, 0, 0, 0);
        const u32x4 as = {sx, 0u, 0u, 0u};
        const u32x4 bs = {sw, 0u, 0u, 0u};
        P = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
    };

    if constexpr (VAR == 0 || VAR == 3) {
        const int wr = wave & 1, wt = wave >> 1;
        const int tok = 32 * wt + c, row = 32 * wr + c;
        i32x16 S0, S1 = im;
        f32x16 P0, P1 = fz;
        i32x4 a0 = rdA(0, tok), b0 = rdB(0, row);
        uint32_t x0 = rdSX(0, tok), w0 = rdSW(0, row);
        auto scaleP = [&](int b, float dw, f32x16 &P) __attribute__((always_inline)) {
            // tokens of the lane's D rows: 8*(i>>2) + 4h + (i&3) -> 4 groups of 4 consecutive fp32
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const f32x4 d = *(const f32x4 *)(sx32 + (b & (R - 1)) * BN + 32 * wt + 8 * g + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; j++) P[4 * g + j] = d[j] * dw;
            }
        };
        for (int b = 0; b < nblk; b += 2) {
            i32x4 a1 = rdA(b + 1, tok), b1 = rdB(b + 1, row);
            uint32_t x1 = rdSX(b + 1, tok), w1 = rdSW(b + 1, row);
            if constexpr (VAR == 0) {
                mfma2(a0, b0, x0, w0, S0, P0);
            } else {
                S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, im, 0, 0, 0);
                scaleP(b, __uint_as_float(w0 | 0x3c000000u), P0);
            }
            epi(acc[0], S1, P1);
            a0 = rdA(b + 2, tok), b0 = rdB(b + 2, row);
            x0 = rdSX(b + 2, tok), w0 = rdSW(b + 2, row);
            if constexpr (VAR == 0) {
                mfma2(a1, b1, x1, w1, S1, P1);
            } else {
                S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, im, 0, 0, 0);
                scaleP(b + 1, __uint_as_float(w1 | 0x3c000000u), P1);
            }
            epi(acc[0], S0, P0);
        }
        epi(acc[0], S1, P1);
    } else if constexpr (VAR == 1 || VAR == 2) {
        // wave = (row tile wr of 2, token pair wt of 2): tiles (wr, 2wt), (wr, 2wt+1); 4 waves cover 64x128
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        for (int b = 0; b < nblk; b++) {
            const i32x4 bb = rdB(b, row);
            const uint32_t w = rdSW(b, row);
            const i32x4 a0 = rdA(b, t0), a1 = rdA(b, t1);
            const uint32_t x0 = rdSX(b, t0), x1 = rdSX(b, t1);
            mfma2(a0, bb, x0, w, S0, P0);
            epi(acc[1], S1, P1);
            if constexpr (VAR == 2) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);   // VALU
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
            }
            mfma2(a1, bb, x1, w, S1, P1);
            epi(acc[0], S0, P0);
            if constexpr (VAR == 2) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 1);
            }
        }
        epi(acc[1], S1, P1);
    } else if constexpr (VAR == 4) {
        // 2 waves cover 64 x 128: wave w takes row tiles 0,1 x token tiles 2w, 2w+1 -> 4 tiles
        const int wt = wave & 1;
        const int tA = 64 * wt + c, tB = 64 * wt + 32 + c;
        i32x16 S[4];
        f32x16 P[4];
#pragma unroll
        for (int t = 0; t < 4; t++) S[t] = im, P[t] = fz;
        for (int b = 0; b < nblk; b++) {
            const i32x4 b0 = rdB(b, c), b1 = rdB(b, 32 + c);
            const uint32_t w0 = rdSW(b, c), w1 = rdSW(b, 32 + c);
            const i32x4 a0 = rdA(b, tA), a1 = rdA(b, tB);
            const uint32_t x0 = rdSX(b, tA), x1 = rdSX(b, tB);
            mfma2(a0, b0, x0, w0, S[0], P[0]);
            epi(acc[2], S[2], P[2]);
            mfma2(a1, b0, x1, w0, S[1], P[1]);
            epi(acc[3], S[3], P[3]);
            mfma2(a0, b1, x0, w1, S[2], P[2]);
            epi(acc[0], S[0], P[0]);
            mfma2(a1, b1, x1, w1, S[3], P[3]);
            epi(acc[1], S[1], P[1]);
        }
        epi(acc[2], S[2], P[2]);
        epi(acc[3], S[3], P[3]);
    }

    if constexpr (VAR == 5) {
        // VAR0 with phases fenced by sched_barrier: the epilogue only touches MFMA results issued a
        // whole phase earlier, operands prefetched one block ahead
        const int wr = wave & 1, wt = wave >> 1;
        const int tok = 32 * wt + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        i32x4 a0 = rdA(0, tok), b0 = rdB(0, row);
        uint32_t x0 = rdSX(0, tok), w0 = rdSW(0, row);
        i32x4 a1 = rdA(1, tok), b1 = rdB(1, row);
        uint32_t x1 = rdSX(1, tok), w1 = rdSW(1, row);
        for (int b = 0; b < nblk; b += 2) {
            mfma2(a0, b0, x0, w0, S0, P0);
            __builtin_amdgcn_sched_barrier(0);
            a0 = rdA(b + 2, tok), b0 = rdB(b + 2, row);
            x0 = rdSX(b + 2, tok), w0 = rdSW(b + 2, row);
            epi(acc[0], S1, P1);
            __builtin_amdgcn_sched_barrier(0);
            mfma2(a1, b1, x1, w1, S1, P1);
            __builtin_amdgcn_sched_barrier(0);
            a1 = rdA(b + 3, tok), b1 = rdB(b + 3, row);
            x1 = rdSX(b + 3, tok), w1 = rdSW(b + 3, row);
            epi(acc[0], S0, P0);
            __builtin_amdgcn_sched_barrier(0);
        }
        epi(acc[0], S1, P1);
    }
    if constexpr (VAR == 6) {
        // VAR1 fenced: mfma(t0,b) | epi(t1,b-1) | mfma(t1,b) | epi(t0,b)
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        for (int b = 0; b < nblk; b++) {
            mfma2(a0, bb, x0, w, S0, P0);
            __builtin_amdgcn_sched_barrier(0);
            epi(acc[1], S1, P1);
            __builtin_amdgcn_sched_barrier(0);
            mfma2(a1, bb, x1, w, S1, P1);
            __builtin_amdgcn_sched_barrier(0);
            bb = rdB(b + 1, row), a0 = rdA(b + 1, t0), a1 = rdA(b + 1, t1);
            w = rdSW(b + 1, row), x0 = rdSX(b + 1, t0), x1 = rdSX(b + 1, t1);
            epi(acc[0], S0, P0);
            __builtin_amdgcn_sched_barrier(0);
        }
        epi(acc[1], S1, P1);
    }
    if constexpr (VAR == 7) {
        const int wt = wave & 1;
        const int tA = 64 * wt + c, tB = 64 * wt + 32 + c;
        i32x16 S[4];
        f32x16 P[4];
#pragma unroll
        for (int t = 0; t < 4; t++) S[t] = im, P[t] = fz;
        i32x4 b0 = rdB(0, c), b1 = rdB(0, 32 + c), a0 = rdA(0, tA), a1 = rdA(0, tB);
        uint32_t w0 = rdSW(0, c), w1 = rdSW(0, 32 + c), x0 = rdSX(0, tA), x1 = rdSX(0, tB);
        for (int b = 0; b < nblk; b++) {
            mfma2(a0, b0, x0, w0, S[0], P[0]);
            __builtin_amdgcn_sched_barrier(0);
            epi(acc[2], S[2], P[2]);
            __builtin_amdgcn_sched_barrier(0);
            mfma2(a1, b0, x1, w0, S[1], P[1]);
            __builtin_amdgcn_sched_barrier(0);
            epi(acc[3], S[3], P[3]);
            __builtin_amdgcn_sched_barrier(0);
            mfma2(a0, b1, x0, w1, S[2], P[2]);
            __builtin_amdgcn_sched_barrier(0);
            mfma2(a1, b1, x1, w1, S[3], P[3]);   // (order: 4 MFMA pairs, epilogues 2 behind)
            __builtin_amdgcn_sched_barrier(0);
            b0 = rdB(b + 1, c), b1 = rdB(b + 1, 32 + c), a0 = rdA(b + 1, tA), a1 = rdA(b + 1, tB);
            w0 = rdSW(b + 1, c), w1 = rdSW(b + 1, 32 + c), x0 = rdSX(b + 1, tA), x1 = rdSX(b + 1, tB);
            epi(acc[0], S[0], P[0]);
            __builtin_amdgcn_sched_barrier(0);
            epi(acc[1], S[1], P[1]);
            __builtin_amdgcn_sched_barrier(0);
        }
        epi(acc[2], S[2], P[2]);
        epi(acc[3], S[3], P[3]);
    }

    if constexpr (VAR == 8) {
        // MFMA only: the same 2 MFMAs per tile-block, 2 tiles per wave, no epilogue
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        const i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        const uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        for (int b = 0; b < nblk; b++) {
            S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bb, S0, 0, 0, 0);
            const u32x4 as = {x0, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u}, as1 = {x1, 0u, 0u, 0u};
            P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as), __builtin_bit_cast(half8, bs), P0, 0, 0, 0);
            S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bb, S1, 0, 0, 0);
            P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), P1, 0, 0, 0);
        }
        epi(acc[0], S0, P0);
        epi(acc[1], S1, P1);
    }
    if constexpr (VAR == 9) {
        // VALU only: the two epilogues per block (32 sub + 32 fma) on fixed S, P
        const int row = c;
        i32x16 S0, S1;
        f32x16 P0, P1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            S0[i] = 0x4B400000 + (int)rdSX(i, row);
            S1[i] = 0x4B400000 + (int)rdSX(i + 3, row);
            P0[i] = 1e-3f * (float)rdSW(i, row);
            P1[i] = 1e-3f * (float)rdSW(i + 1, row);
        }
        for (int b = 0; b < nblk; b++) {
            epi(acc[0], S0, P0);
            epi(acc[1], S1, P1);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if constexpr (VAR == 10) {
        // VAR1 with the i8 MFMA accumulating on 0 (inline C) and v_cvt_f32_i32 in the epilogue
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        const i32x16 iz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        i32x16 S0 = iz, S1 = iz;
        f32x16 P0 = fz, P1 = fz;
        auto epc = [&](float *a, const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = fmaf((float)S[i], P[i], a[i]);
        };
        for (int b = 0; b < nblk; b++) {
            const i32x4 bb = rdB(b, row);
            const uint32_t w = rdSW(b, row);
            const i32x4 a0 = rdA(b, t0), a1 = rdA(b, t1);
            const uint32_t x0 = rdSX(b, t0), x1 = rdSX(b, t1);
            S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bb, iz, 0, 0, 0);
            {
                const u32x4 as = {x0, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u};
                P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
            }
            epc(acc[1], S1, P1);
            S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bb, iz, 0, 0, 0);
            {
                const u32x4 as = {x1, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u};
                P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
            }
            epc(acc[0], S0, P0);
        }
        epc(acc[1], S1, P1);
    }

    if constexpr (VAR == 12 || VAR == 13) {
        // 12: MFMA chains (as VAR 8) + the epilogue VALU on registers no MFMA writes, in one wave
        // 13: blockIdx parity picks the role: even workgroups MFMA only, odd VALU only (2 WG/CU ->
        //     one MFMA wave and one VALU wave per SIMD)
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        const i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        const uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        i32x16 Q0, Q1;
        f32x16 R0, R1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            Q0[i] = 0x4B400000 + (int)rdSX(i, row);
            Q1[i] = 0x4B400000 + (int)rdSX(i + 3, row);
            R0[i] = 1e-3f * (float)rdSW(i, row);
            R1[i] = 1e-3f * (float)rdSW(i + 1, row);
        }
        const bool do_m = VAR == 12 || !(blockIdx.x & 1), do_v = VAR == 12 || (blockIdx.x & 1);
        const u32x4 as = {x0, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u}, as1 = {x1, 0u, 0u, 0u};
        for (int b = 0; b < nblk; b++) {
            if (do_m) {
                S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bb, S0, 0, 0, 0);
                P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as), __builtin_bit_cast(half8, bs), P0, 0, 0, 0);
            }
            if (do_v) epi(acc[0], Q0, R0);
            if (do_m) {
                S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bb, S1, 0, 0, 0);
                P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), P1, 0, 0, 0);
            }
            if (do_v) epi(acc[1], Q1, R1);
        }
        epi(acc[2], S0, P0);
        epi(acc[3], S1, P1);
    }

    if constexpr (VAR == 14 || VAR == 24) {
        // 1 tile/wave, (S, P) ring of 3: the epilogue consumes the MFMAs of two blocks back
        constexpr bool F = VAR == 24;
        const int wr = wave & 1, wt = wave >> 1;
        const int tok = 32 * wt + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im, S2 = im;
        f32x16 P0 = fz, P1 = fz, P2 = fz;
        i32x4 a = rdA(0, tok), bb = rdB(0, row);
        uint32_t x = rdSX(0, tok), w = rdSW(0, row);
        auto step = [&](int b, i32x16 &Sn, f32x16 &Pn, i32x16 &So, f32x16 &Po) __attribute__((always_inline)) {
            mfma2(a, bb, x, w, Sn, Pn);
            if (F) __builtin_amdgcn_sched_barrier(0);
            a = rdA(b + 1, tok), bb = rdB(b + 1, row);
            x = rdSX(b + 1, tok), w = rdSW(b + 1, row);
            epi(acc[0], So, Po);
            if (F) __builtin_amdgcn_sched_barrier(0);
        };
        for (int b = 0; b < nblk; b += 3) {
            step(b, S0, P0, S1, P1);
            step(b + 1, S1, P1, S2, P2);
            step(b + 2, S2, P2, S0, P0);
        }
        epi(acc[0], S1, P1);
        epi(acc[0], S2, P2);
    }
    if constexpr (VAR == 15 || VAR == 25) {
        // 2 tiles/wave, 2 (S, P) sets per tile: M(t0,b) M(t1,b) E(t0,b-1) E(t1,b-1)
        constexpr bool F = VAR == 25;
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 SA0 = im, SA1 = im, SB0 = im, SB1 = im;
        f32x16 PA0 = fz, PA1 = fz, PB0 = fz, PB1 = fz;
        i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        auto step = [&](int b, i32x16 &Sa, f32x16 &Pa, i32x16 &Sb, f32x16 &Pb, i32x16 &Sa_, f32x16 &Pa_,
                        i32x16 &Sb_, f32x16 &Pb_) __attribute__((always_inline)) {
            mfma2(a0, bb, x0, w, Sa, Pa);
            mfma2(a1, bb, x1, w, Sb, Pb);
            if (F) __builtin_amdgcn_sched_barrier(0);
            bb = rdB(b + 1, row), a0 = rdA(b + 1, t0), a1 = rdA(b + 1, t1);
            w = rdSW(b + 1, row), x0 = rdSX(b + 1, t0), x1 = rdSX(b + 1, t1);
            epi(acc[0], Sa_, Pa_);
            epi(acc[1], Sb_, Pb_);
            if (F) __builtin_amdgcn_sched_barrier(0);
        };
        for (int b = 0; b < nblk; b += 2) {
            step(b, SA0, PA0, SB0, PB0, SA1, PA1, SB1, PB1);
            step(b + 1, SA1, PA1, SB1, PB1, SA0, PA0, SB0, PB0);
        }
        epi(acc[0], SA1, PA1);
        epi(acc[1], SB1, PB1);
    }

    if constexpr (VAR == 16 || VAR == 17) {
        // VAR15 structure; 16: operands fixed (no LDS reads in the loop); 17: LDS reads kept but the
        // epilogue reads registers no MFMA writes (as VAR 12)
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 SA0 = im, SA1 = im, SB0 = im, SB1 = im;
        f32x16 PA0 = fz, PA1 = fz, PB0 = fz, PB1 = fz;
        i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        i32x16 Q0, Q1;
        f32x16 R0, R1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            Q0[i] = 0x4B400000 + (int)rdSX(i, row);
            Q1[i] = 0x4B400000 + (int)rdSX(i + 3, row);
            R0[i] = 1e-3f * (float)rdSW(i, row);
            R1[i] = 1e-3f * (float)rdSW(i + 1, row);
        }
        auto step = [&](int b, i32x16 &Sa, f32x16 &Pa, i32x16 &Sb, f32x16 &Pb, i32x16 &Sa_, f32x16 &Pa_,
                        i32x16 &Sb_, f32x16 &Pb_) __attribute__((always_inline)) {
            mfma2(a0, bb, x0, w, Sa, Pa);
            mfma2(a1, bb, x1, w, Sb, Pb);
            if (VAR == 17) {
                bb = rdB(b + 1, row), a0 = rdA(b + 1, t0), a1 = rdA(b + 1, t1);
                w = rdSW(b + 1, row), x0 = rdSX(b + 1, t0), x1 = rdSX(b + 1, t1);
                epi(acc[0], Q0, R0);
                epi(acc[1], Q1, R1);
            } else {
                epi(acc[0], Sa_, Pa_);
                epi(acc[1], Sb_, Pb_);
            }
        };
        for (int b = 0; b < nblk; b += 2) {
            step(b, SA0, PA0, SB0, PB0, SA1, PA1, SB1, PB1);
            step(b + 1, SA1, PA1, SB1, PB1, SA0, PA0, SB0, PB0);
        }
        epi(acc[2], SA1, PA1);
        epi(acc[3], SB1, PB1);
        epi(acc[2], SA0, PA0);
        epi(acc[3], SB0, PB0);
    }

    if constexpr (VAR == 18) {
        // VAR15 with the MFMAs spread through the epilogue VALU by sched_group_barrier:
        // [MFMA, 18 VALU] x 4, the next block's LDS reads after the second MFMA
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 SA0 = im, SA1 = im, SB0 = im, SB1 = im;
        f32x16 PA0 = fz, PA1 = fz, PB0 = fz, PB1 = fz;
        i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        auto step = [&](int b, i32x16 &Sa, f32x16 &Pa, i32x16 &Sb, f32x16 &Pb, i32x16 &Sa_, f32x16 &Pa_,
                        i32x16 &Sb_, f32x16 &Pb_) __attribute__((always_inline)) {
            mfma2(a0, bb, x0, w, Sa, Pa);
            mfma2(a1, bb, x1, w, Sb, Pb);
            bb = rdB(b + 1, row), a0 = rdA(b + 1, t0), a1 = rdA(b + 1, t1);
            w = rdSW(b + 1, row), x0 = rdSX(b + 1, t0), x1 = rdSX(b + 1, t1);
            epi(acc[0], Sa_, Pa_);
            epi(acc[1], Sb_, Pb_);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
        };
        for (int b = 0; b < nblk; b += 2) {
            step(b, SA0, PA0, SB0, PB0, SA1, PA1, SB1, PB1);
            step(b + 1, SA1, PA1, SB1, PB1, SA0, PA0, SB0, PB0);
        }
        epi(acc[0], SA1, PA1);
        epi(acc[1], SB1, PB1);
    }
    if constexpr (VAR == 19) {
        // 1 tile/wave, ring of 3, [MFMA, 18 VALU] x 2 per block
        const int wr = wave & 1, wt = wave >> 1;
        const int tok = 32 * wt + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im, S2 = im;
        f32x16 P0 = fz, P1 = fz, P2 = fz;
        i32x4 a = rdA(0, tok), bb = rdB(0, row);
        uint32_t x = rdSX(0, tok), w = rdSW(0, row);
        auto step = [&](int b, i32x16 &Sn, f32x16 &Pn, i32x16 &So, f32x16 &Po) __attribute__((always_inline)) {
            mfma2(a, bb, x, w, Sn, Pn);
            a = rdA(b + 1, tok), bb = rdB(b + 1, row);
            x = rdSX(b + 1, tok), w = rdSW(b + 1, row);
            epi(acc[0], So, Po);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 18, 0);
        };
        for (int b = 0; b < nblk; b += 3) {
            step(b, S0, P0, S1, P1);
            step(b + 1, S1, P1, S2, P2);
            step(b + 2, S2, P2, S0, P0);
        }
        epi(acc[0], S1, P1);
        epi(acc[0], S2, P2);
    }

    if constexpr (VAR == 21 || VAR == 22) {
        // VAR1 structure with (a) loop-carried scale operands (only element 0 rewritten, no v_and /
        // v_mov rebuild: d_x read as the raw dword {sx_b, sx_b+1}, whose upper half meets B's zero k=1),
        // (b) 22: the epilogue in packed f32 (v_pk_add_f32 / v_pk_fma_f32, 2 outputs per instruction)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 S0 = im, S1 = im;
        f32x16 P0 = fz, P1 = fz;
        u32x4 as0 = {0u, 0u, 0u, 0u}, as1 = {0u, 0u, 0u, 0u}, bs = {0u, 0u, 0u, 0u};
        const uint32_t *sx32w = (const uint32_t *)sx16;
        auto epi2 = [&](float *a, const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
            if constexpr (VAR == 22) {
                const f32x2 bias = {-12582912.0f, -12582912.0f};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    f32x2 sv = {__int_as_float(S[i]), __int_as_float(S[i + 1])};
                    f32x2 pv = {P[i], P[i + 1]};
                    f32x2 av = {a[i], a[i + 1]};
                    sv = sv + bias;
                    av = __builtin_elementwise_fma(sv, pv, av);
                    a[i] = av.x;
                    a[i + 1] = av.y;
                }
            } else {
                epi(a, S, P);
            }
        };
        for (int b = 0; b < nblk; b++) {
            const i32x4 bb = rdB(b, row);
            bs.x = rdSW(b, row);
            const i32x4 a0 = rdA(b, t0), a1 = rdA(b, t1);
            as0.x = sx32w[((b & (R - 1)) * BN + t0) >> 1];
            as1.x = sx32w[((b & (R - 1)) * BN + t1) >> 1];
            S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bb, im, 0, 0, 0);
            P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as0), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
            epi2(acc[1], S1, P1);
            S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bb, im, 0, 0, 0);
            P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
            epi2(acc[0], S0, P0);
        }
        epi2(acc[1], S1, P1);
    }

    if constexpr (VAR == 30 || VAR == 31 || VAR == 32) {
        // 30: MFMA only, C = constant (im / 0), fresh destinations (the GEMM's form) — vs VAR 8 (chained)
        // 31: VAR 16 (2 sets, epilogue reads the other set) but the MFMAs accumulate in place (D = C)
        // 32: VAR 16 exactly, for reference (no LDS)
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 SA0 = im, SA1 = im, SB0 = im, SB1 = im;
        f32x16 PA0 = fz, PA1 = fz, PB0 = fz, PB1 = fz;
        const i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        const uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        const u32x4 as = {x0, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u}, as1 = {x1, 0u, 0u, 0u};
        auto mf = [&](const i32x4 &a, const u32x4 &sx, i32x16 &S, f32x16 &P) __attribute__((always_inline)) {
            if constexpr (VAR == 31) {
                S = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bb, S, 0, 0, 0);
                P = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, sx), __builtin_bit_cast(half8, bs), P, 0, 0, 0);
            } else {
                S = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bb, im, 0, 0, 0);
                P = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, sx), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
            }
        };
        auto step = [&](i32x16 &Sa, f32x16 &Pa, i32x16 &Sb, f32x16 &Pb, i32x16 &Sa_, f32x16 &Pa_, i32x16 &Sb_,
                        f32x16 &Pb_) __attribute__((always_inline)) {
            mf(a0, as, Sa, Pa);
            mf(a1, as1, Sb, Pb);
            if constexpr (VAR != 30) {
                epi(acc[0], Sa_, Pa_);
                epi(acc[1], Sb_, Pb_);
            }
        };
        for (int b = 0; b < nblk; b += 2) {
            step(SA0, PA0, SB0, PB0, SA1, PA1, SB1, PB1);
            step(SA1, PA1, SB1, PB1, SA0, PA0, SB0, PB0);
        }
        epi(acc[2], SA1, PA1);
        epi(acc[3], SB1, PB1);
        epi(acc[2], SA0, PA0);
        epi(acc[3], SB0, PB0);
    }

    if constexpr (VAR == 33) {
        // VAR 32 with the MFMAs as inline asm writing AGPRs (acc file); the epilogue reads them through
        // v_accvgpr_read (compiler-inserted), results consumed two bursts later (wait states long met)
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        i32x16 SA0 = {}, SA1 = {}, SB0 = {}, SB1 = {};
        f32x16 PA0 = fz, PA1 = fz, PB0 = fz, PB1 = fz;
        const i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        const uint32_t w = rdSW(0, row), x0 = rdSX(0, t0), x1 = rdSX(0, t1);
        const u32x4 as = {x0, 0u, 0u, 0u}, bs = {w, 0u, 0u, 0u}, as1 = {x1, 0u, 0u, 0u};
        auto mf = [&](const i32x4 &a, const u32x4 &sx, i32x16 &S, f32x16 &P) __attribute__((always_inline)) {
            asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %2, 0" : "=a"(S) : "v"(a), "v"(bb));
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=a"(P) : "v"(sx), "v"(bs));
        };
        auto epc = [&](float *acc_, const i32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 16; i++) acc_[i] = fmaf((float)S[i], P[i], acc_[i]);
        };
        auto step = [&](i32x16 &Sa, f32x16 &Pa, i32x16 &Sb, f32x16 &Pb, i32x16 &Sa_, f32x16 &Pa_, i32x16 &Sb_,
                        f32x16 &Pb_) __attribute__((always_inline)) {
            mf(a0, as, Sa, Pa);
            mf(a1, as1, Sb, Pb);
            epc(acc[0], Sa_, Pa_);
            epc(acc[1], Sb_, Pb_);
        };
        for (int b = 0; b < nblk; b += 2) {
            step(SA0, PA0, SB0, PB0, SA1, PA1, SB1, PB1);
            step(SA1, PA1, SB1, PB1, SA0, PA0, SB0, PB0);
        }
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
        epc(acc[2], SA1, PA1);
        epc(acc[3], SB1, PB1);
    }

    if constexpr (VAR == 35) {
        // scale product on the VALU (P = d_x * d_w from fp32 LDS values: no scale MFMA), and the
        // MFMA results drained (int -> float) BEFORE the next block's MFMAs are issued, so that the
        // VALU that overlaps the MFMA burst (the P products and the fmas) reads no MFMA-written register
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        const i32x16 iz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        i32x16 S0 = iz, S1 = iz;
        float F0[16], F1[16];
        i32x4 bb = rdB(0, row), a0 = rdA(0, t0), a1 = rdA(0, t1);
        for (int b = 0; b < nblk; b++) {
            // drain the previous block's sums (the wave waits here once for its burst)
#pragma unroll
            for (int i = 0; i < 16; i++) F0[i] = (float)S0[i], F1[i] = (float)S1[i];
            __builtin_amdgcn_sched_barrier(0);
            S0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, bb, iz, 0, 0, 0);
            S1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, bb, iz, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            // next operands + this (previous) block's scales, then the fmas
            const float dw = __uint_as_float(0x3a000000u | rdSW(b - 1, row));
            const float *xd = sx32 + ((b - 1) & (R - 1)) * BN;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const f32x4 d0 = *(const f32x4 *)(xd + 64 * wt + 8 * g + 4 * h);
                const f32x4 d1 = *(const f32x4 *)(xd + 64 * wt + 32 + 8 * g + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[0][4 * g + j] = fmaf(F0[4 * g + j], d0[j] * dw, acc[0][4 * g + j]);
                    acc[1][4 * g + j] = fmaf(F1[4 * g + j], d1[j] * dw, acc[1][4 * g + j]);
                }
            }
            bb = rdB(b + 1, row), a0 = rdA(b + 1, t0), a1 = rdA(b + 1, t1);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) acc[2][i] += (float)S0[i] + (float)S1[i];
    }

    if constexpr (VAR == 36 || VAR == 37 || VAR == 38 || VAR == 39 || VAR == 40 || VAR == 41) {
        // VAR21 with the block sum from the block-scaled fp6 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4,
        // e2m3 operands: w/2 and [x_hi/2 | x_lo/2] with power-of-two block scales -> the exact integer
        // sum as an f32, no conversion in the epilogue): 36 with the epilogue, 37 MFMAs only
        typedef int i32x8 __attribute__((ext_vector_type(8)));
        const int wr = wave & 1, wt = (wave >> 1) & 1;
        const int t0 = 64 * wt + c, t1 = 64 * wt + 32 + c, row = 32 * wr + c;
        f32x16 S0 = fz, S1 = fz;
        f32x16 P0 = fz, P1 = fz;
        u32x4 as0 = {0u, 0u, 0u, 0u}, as1 = {0u, 0u, 0u, 0u}, bs = {0u, 0u, 0u, 0u};
        const uint32_t *sx32w = (const uint32_t *)sx16;
        auto rd6 = [&](int off) __attribute__((always_inline)) {
            const i32x4 u = *(const i32x4 *)(lds + off);
            const int2 v = *(const int2 *)(lds + off + 16);
            const i32x8 r = {u.x, u.y, u.z, u.w, v.x, v.y, 0, 0};
            return r;
        };
        auto epi3 = [&](float *a, const f32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = fmaf(S[i], P[i], a[i]);
        };
        const int sa = 128, sb = VAR == 40 ? (h ? 128 : 132) : 127 + 4;
        for (int b = 0; b < nblk; b++) {
            const int rb = (b & (R - 1));
            const i32x8 bb = rd6(LA + rb * BM * 32 + (row & 15) * 48 + 24 * h);
            bs.x = rdSW(b, row);
            const i32x8 a0 = rd6(rb * BN * 32 + (t0 & 31) * 96 + 48 * h);
            const i32x8 a1 = rd6(rb * BN * 32 + (t1 & 31) * 96 + 48 * h + 3072);
            as0.x = sx32w[(rb * BN + t0) >> 1];
            as1.x = sx32w[(rb * BN + t1) >> 1];
            if constexpr (VAR == 36 || VAR == 40) {
                S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, fz, 2, 2, 0, sb, 0, sa);
                P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as0), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
                epi3(acc[1], S1, P1);
                S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, fz, 2, 2, 0, sb, 0, sa);
                P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
                epi3(acc[0], S0, P0);
            } else if constexpr (VAR == 41) {          // VAR36 with the roles of A and B swapped (B shared)
                S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bb, a0, fz, 2, 2, 0, sa, 0, sb);
                P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as0), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
                epi3(acc[1], S1, P1);
                S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bb, a1, fz, 2, 2, 0, sa, 0, sb);
                P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), fz, 0, 0, 0);
                epi3(acc[0], S0, P0);
            } else if constexpr (VAR == 38) {          // fp6 only, 4 chains
                S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, S0, 2, 2, 0, sb, 0, sa);
                S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, S1, 2, 2, 0, sb, 0, sa);
                P0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, P0, 2, 2, 0, sb, 0, sa);
                P1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, P1, 2, 2, 0, sb, 0, sa);
            } else if constexpr (VAR == 39) {          // i8 only, 4 chains
                i32x16 *SI = (i32x16 *)&S0, *SJ = (i32x16 *)&S1, *PI = (i32x16 *)&P0, *PJ = (i32x16 *)&P1;
                const i32x4 x0 = {a0.x, a0.y, a0.z, a0.w}, x1 = {a1.x, a1.y, a1.z, a1.w}, w4 = {bb.x, bb.y, bb.z, bb.w};
                *SI = __builtin_amdgcn_mfma_i32_32x32x32_i8(x0, w4, *SI, 0, 0, 0);
                *SJ = __builtin_amdgcn_mfma_i32_32x32x32_i8(x1, w4, *SJ, 0, 0, 0);
                *PI = __builtin_amdgcn_mfma_i32_32x32x32_i8(x0, w4, *PI, 0, 0, 0);
                *PJ = __builtin_amdgcn_mfma_i32_32x32x32_i8(x1, w4, *PJ, 0, 0, 0);
            } else {
                S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, S0, 2, 2, 0, sb, 0, sa);
                P0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as0), __builtin_bit_cast(half8, bs), P0, 0, 0, 0);
                S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, S1, 2, 2, 0, sb, 0, sa);
                P1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, as1), __builtin_bit_cast(half8, bs), P1, 0, 0, 0);
            }
        }
        if constexpr (VAR == 36 || VAR == 40 || VAR == 41) {
            epi3(acc[1], S1, P1);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) acc[0][i] += S0[i] + S1[i] + P0[i] + P1[i];
        }
    }
    if constexpr (VAR >= 42 && VAR <= 45) {
        // issue rate of one instruction kind, four independent accumulator chains per wave:
        // 42 v_mfma_f32_32x32x16_f16 (the scale product's), 43 v_mfma_f32_32x32x8_f16 (legacy form),
        // 44 the block-scaled f8f6f4 MFMA with fp4 (e2m1) operands, 45 with fp8 (e4m3) operands
        typedef int i32x8 __attribute__((ext_vector_type(8)));
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        f32x16 C0 = fz, C1 = fz, C2 = fz, C3 = fz;
        for (int b = 0; b < nblk; b++) {
            const int rb = (b & (R - 1));
            const i32x4 u = *(const i32x4 *)(lds + rb * BN * 32 + c * 16);
            const i32x4 v = *(const i32x4 *)(lds + LA + rb * BM * 32 + c * 16);
            if constexpr (VAR == 42) {
                const half8 a = __builtin_bit_cast(half8, u), bb = __builtin_bit_cast(half8, v);
                C0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bb, C0, 0, 0, 0);
                C1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb, a, C1, 0, 0, 0);
                C2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, a, C2, 0, 0, 0);
                C3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb, bb, C3, 0, 0, 0);
            } else if constexpr (VAR == 43) {
                const int2 u2 = {u.x, u.y}, v2 = {v.x, v.y};
                const half4 a = __builtin_bit_cast(half4, u2), bb = __builtin_bit_cast(half4, v2);
                C0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a, bb, C0, 0, 0, 0);
                C1 = __builtin_amdgcn_mfma_f32_32x32x8f16(bb, a, C1, 0, 0, 0);
                C2 = __builtin_amdgcn_mfma_f32_32x32x8f16(a, a, C2, 0, 0, 0);
                C3 = __builtin_amdgcn_mfma_f32_32x32x8f16(bb, bb, C3, 0, 0, 0);
            } else {
                constexpr int F = VAR == 44 ? 4 : 0;
                const i32x8 a = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w}, bb = {v.x, v.y, v.z, v.w, u.x, u.y, u.z, u.w};
                C0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, C0, F, F, 0, 127, 0, 127);
                C1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bb, a, C1, F, F, 0, 127, 0, 127);
                C2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, C2, F, F, 0, 127, 0, 127);
                C3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bb, bb, C3, F, F, 0, 127, 0, 127);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) acc[0][i] += C0[i] + C1[i] + C2[i] + C3[i];
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int i = 0; i < 16; i++) s += acc[t][i];
    out[blockIdx.x * 512 + tid] = s;
}

template <int VAR>
void run(const char *name, int waves, int tiles_per_wave, const uint8_t *src, float *out, int nblk, int wg_per_cu) {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int grid = cus * wg_per_cu;
    CK(hipFuncSetAttribute((const void *)k_mb<VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k_mb<VAR>, dim3(grid), dim3(waves * 64), LDS, 0, src, out, nblk);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k_mb<VAR>, dim3(grid), dim3(waves * 64), LDS, 0, src, out, nblk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    // tile-blocks per SIMD: grid * waves * tiles * nblk / (cus * 4)
    const double tb = (double)grid * waves * tiles_per_wave * nblk / (cus * 4.0);
    const double ops = 2.0 * 32 * 32 * 32 * grid * waves * tiles_per_wave * (double)nblk;
    printf("%-44s waves/WG %2d WG/CU %d: %8.2f us  %6.1f cyc/(tile*blk)/SIMD @2.4GHz  %6.1f TOP/s\n", name, waves, wg_per_cu,
           us, us * 2400.0 / tb, ops / us * 1e-6);
}

int main(int argc, char **argv) {
    const int nblk = argc > 1 ? atoi(argv[1]) : 2048;
    const int fill = argc > 2 ? atoi(argv[2]) : 0;     // 0 hash bytes, 1 zeros, 2 0x41 bytes, 3 0x08 bytes
    std::vector<uint8_t> h(LDS);
    for (size_t i = 0; i < h.size(); i++)
        h[i] = fill == 1 ? 0 : fill == 2 ? 0x41 : fill == 3 ? 0x08 : (uint8_t)((i * 2654435761u) >> 13);
    uint8_t *src;
    float *out;
    CK(hipMalloc(&src, LDS));
    CK(hipMalloc(&out, 4096 * 512 * 4));
    CK(hipMemcpy(src, h.data(), LDS, hipMemcpyHostToDevice));
    // waves per SIMD = waves/WG x WG/CU / 4 where registers allow
    printf("fill %d\n", fill);
    run<21>("VAR21 i8 2 tiles/wave (gemm8 structure)", 4, 2, src, out, nblk, 2);
    run<36>("VAR36 fp6 block sum, f32 epilogue (no cvt)", 4, 2, src, out, nblk, 2);
    run<38>("VAR38 fp6 x2 per tile-blk, 4 chains", 4, 2, src, out, nblk, 2);
    if (argc > 3) {        // instruction issue rates: 4 MFMAs per block-step, reported per MFMA (x2 tiles)
        run<39>("VAR39 i8 32x32x32, 4 chains", 4, 2, src, out, nblk, 2);
        run<42>("VAR42 f16 32x32x16, 4 chains", 4, 2, src, out, nblk, 2);
        run<43>("VAR43 f16 32x32x8 (legacy), 4 chains", 4, 2, src, out, nblk, 2);
        run<44>("VAR44 fp4 32x32x64 (scale), 4 chains", 4, 2, src, out, nblk, 2);
        run<45>("VAR45 fp8 32x32x64 (scale), 4 chains", 4, 2, src, out, nblk, 2);
        run<42>("VAR42 f16 32x32x16, 4 chains", 4, 2, src, out, nblk, 1);
        run<44>("VAR44 fp4 32x32x64 (scale), 4 chains", 4, 2, src, out, nblk, 1);
    }
    return 0;
}
