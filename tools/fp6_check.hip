// Exactness and operand-layout check of the block-scaled fp6 MFMA as an exact q4_0 x q8_0 block sum
// (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 operands): for 32 rows of q4_0 weights w in [-8, 7] and 32
// tokens of q8_0 values x in [-128, 127], one instruction with
//   A (weights)  lane r + 32h: the 32 values w/2 of row r (both lane halves), block scale 2^1
//   B (x)        lane t + 32h: h = 0 -> the 32 values (x >> 4)/2, scale 2^5; h = 1 -> (x & 15)/2, scale 2^1
// computes sum_k w*(16*(x >> 4) + (x & 15)) = sum_k w*x exactly (every partial sum an integer < 2^24).
// Prints the number of mismatching outputs over many random trials and the layout found.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

// e2m3 code of v = n/2, n an integer in [-15, 15] (|v| <= 7.5, a multiple of 0.5)
static uint32_t e2m3_half(int n) {
    const uint32_t s = n < 0 ? 0x20u : 0u;
    const int a = n < 0 ? -n : n;            // |v| = a/2, in eighths: 4a
    const int e8 = 4 * a;                    // |v| * 8
    uint32_t code;
    if (e8 < 8) code = (uint32_t)e8;                              // e = 0: m/8
    else if (e8 < 16) code = (1u << 3) | (uint32_t)(e8 - 8);      // e = 1: 1 + m/8
    else if (e8 < 32) code = (2u << 3) | (uint32_t)((e8 - 16) / 2);   // e = 2: 2(1 + m/8)
    else code = (3u << 3) | (uint32_t)((e8 - 32) / 4);                // e = 3: 4(1 + m/8)
    return s | code;
}

// pack 32 6-bit codes into 6 dwords, element j at bits [6j, 6j + 6)
static void pack6(const uint32_t *c, uint32_t *o) {
    for (int i = 0; i < 6; i++) o[i] = 0;
    for (int j = 0; j < 32; j++) {
        const int bit = 6 * j;
        o[bit >> 5] |= c[j] << (bit & 31);
        if ((bit & 31) > 26) o[(bit >> 5) + 1] |= c[j] >> (32 - (bit & 31));
    }
}

__global__ void k_fp6(const uint32_t *A, const uint32_t *B, float *D, int trials) {
    const int l = threadIdx.x;
    for (int t = 0; t < trials; t++) {
        i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 6; i++) {
            a[i] = (int)A[((size_t)t * 64 + l) * 6 + i];
            b[i] = (int)B[((size_t)t * 64 + l) * 6 + i];
        }
        const int sa = 128, sb = (l >> 5) ? 128 : 132;
        const f32x16 z = {};
        const f32x16 d = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, z, 2, 2, 0, sa, 0, sb);
        for (int i = 0; i < 16; i++) D[((size_t)t * 64 + l) * 16 + i] = d[i];
    }
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 256;
    std::vector<int> w((size_t)trials * 32 * 32), x((size_t)trials * 32 * 32);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (size_t i = 0; i < w.size(); i++) {
        w[i] = (int)(rnd() % 16) - 8;
        x[i] = (int)(rnd() % 256) - 128;
        if (i < 64 * 32) x[i] = (i & 1) ? 127 : -128, w[i] = (i & 2) ? 7 : -8;      // extremes in trial 0
    }
    // A: lane r + 32h holds w[row r][k], k = 0..31 (both halves); B: lane c + 32h holds x parts of token c
    std::vector<uint32_t> hA((size_t)trials * 64 * 6), hB((size_t)trials * 64 * 6);
    for (int t = 0; t < trials; t++)
        for (int l = 0; l < 64; l++) {
            const int r = l & 31, h = l >> 5;
            uint32_t ca[32], cb[32];
            for (int k = 0; k < 32; k++) {
                ca[k] = e2m3_half(w[((size_t)t * 32 + r) * 32 + k]);
                const int xv = x[((size_t)t * 32 + r) * 32 + k];
                cb[k] = e2m3_half(h ? (xv & 15) : (xv >> 4));
            }
            pack6(ca, &hA[((size_t)t * 64 + l) * 6]);
            pack6(cb, &hB[((size_t)t * 64 + l) * 6]);
        }
    uint32_t *dA, *dB;
    float *dD;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB, hB.size() * 4));
    CK(hipMalloc(&dD, (size_t)trials * 64 * 16 * 4));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fp6, dim3(1), dim3(64), 0, 0, dA, dB, dD, trials);
    CK(hipDeviceSynchronize());
    std::vector<float> hD((size_t)trials * 64 * 16);
    CK(hipMemcpy(hD.data(), dD, hD.size() * 4, hipMemcpyDeviceToHost));
    // D layout (shape-determined): lane l, reg i -> row (i&3) + 8(i>>2) + 4(l>>5) of A, column l&31 of B
    long bad = 0, badT = 0;
    for (int t = 0; t < trials; t++)
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 16; i++) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
                long ref = 0, refT = 0;
                for (int k = 0; k < 32; k++) {
                    ref += (long)w[((size_t)t * 32 + row) * 32 + k] * x[((size_t)t * 32 + col) * 32 + k];
                    refT += (long)w[((size_t)t * 32 + col) * 32 + k] * x[((size_t)t * 32 + row) * 32 + k];
                }
                const float g = hD[((size_t)t * 64 + l) * 16 + i];
                if (g != (float)ref) {
                    if (bad < 5) printf("mismatch t=%d lane=%d reg=%d: got %.1f want %ld (transposed %ld)\n", t, l, i, g, ref, refT);
                    bad++;
                }
                if (g != (float)refT) badT++;
            }
    printf("fp6 block-scaled MFMA as exact block sum: %d trials x 1024 outputs, mismatches %ld (row=A,col=B), %ld (transposed)\n",
           trials, bad, badT);
    return bad ? 1 : 0;
}
