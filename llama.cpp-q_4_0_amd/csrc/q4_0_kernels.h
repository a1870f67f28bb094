// q4_0_kernels.h — launchers for the gfx950 q4_0 x q8_0 kernels (internal to libggml_hip.so).
//
// Data layouts in HBM:
//   W   : ggml block_q4_0 rows, verbatim (ggml.c:870-875): row m at W + m*rowbytes,
//         rowbytes = 18*K/32; block = fp16 d + 16 bytes of nibbles (elem j: low nibble
//         of qs[j], elem j+16: high nibble).  Never repacked.
//   x   : f32 [N][K] (ggml src1, nb10 == 4).
//   y   : f32 [N][ldy] (ggml dst, y[n*ldy + m]).
//   xq8 : ggml block_q8_0 rows (ggml.c:902-907), AoS, 34*K/32 bytes per token — the
//         reference's INIT wdata layout; produced by quantize_q8_0_aos.
//   xs  : internal GEMM operand: int8 qs [N][K] + f32 d [N][K/32] (fp32 value of the
//         fp16-rounded scale), produced by quantize_q8_0_soa from the same device
//         quantizer; bit-identical q8_0 values.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghip {

struct DeviceInfo {
    int num_cus;
};

// A5 (AVX2 branch semantics, bit-exact): x f32 [N][K] -> block_q8_0 AoS [N][K/32].
hipError_t quantize_q8_0_aos(const float *x, int64_t K, int64_t N, void *xq8, hipStream_t s);
// Same quantizer, GEMM operand layout.
hipError_t quantize_q8_0_soa(const float *x, int64_t K, int64_t N, int8_t *qs, float *d, hipStream_t s,
                             uint16_t *d16 = nullptr);   // d16: optional fp16 copy of d, block-major [K/32][N]
// A3 (quantize_row_q4_0_reference semantics, bit-exact): w f32 [M][K] -> block_q4_0 rows.
hipError_t quantize_q4_0(const float *w, int64_t K, int64_t M, void *wq, hipStream_t s);
// A4: block_q4_0 rows -> f32 [M][K].
hipError_t dequantize_q4_0(const void *wq, int64_t K, int64_t M, float *w, hipStream_t s);

// Decode / small-batch path: fused q8_0 quantize of x (in LDS) + q4_0.q8_0 GEMV.
// N <= gemv_max_tokens(K).
int gemv_max_tokens(int64_t K);
hipError_t gemv_q4_0(const void *W, int64_t K, int64_t M, const float *x, int64_t N,
                     float *y, int64_t ldy, const DeviceInfo &dev, hipStream_t s);

// Sibling mul_mats sharing x (e.g. wq/wk/wv): up to 4 matrices of the same K in one launch.
constexpr int GEMV_MULTI_MAX = 4;
hipError_t gemv_q4_0_multi(int nmat, const void *const *W, const int64_t *M, int64_t K, const float *x, int64_t N,
                           float *const *y, const int64_t *ldy, const DeviceInfo &dev, hipStream_t s);

// The same for N = 1 with the chain that produces x folded into the x prologue (K <= 16384); the
// GEMVs consume x, and workgroup 0 also stores the chain's tensors (each may be null) bit for bit as
// the unfused launches:
//   kind 1, ggml's [add ->] rms_norm -> mul(norm weight row): x = (a ? a + b : b) -> sum,
//           x *= 1/sqrt(mean(x*x) + 1e-6) (double sum, as ggml_ops.hip's k_row_norm4) -> norm,
//           x *= w -> out;
//   kind 2, silu -> mul: u = fp16 table[fp16(a)] (ggml's GGML_SILU_FP16) -> norm, x = u * b -> out.
struct GemvNorm {
    const float *a, *w;
    float *sum, *norm, *out;
    int kind = 1;
    const uint16_t *table = nullptr;     // kind 2: ggml's silu table (65536 fp16 bit patterns)
};
// Decode epilogue of a sibling GEMV (hook path, one token): the elementwise nodes ggml emits right after the
// q|k|v mul_mats (rope mode 0 of K and Q in place, K into the K cache, V into the transposed V cache) done by
// the GEMV on its own output element e of matrix i, with the arithmetic of k_elem_batch (ggml_ops.hip) bit
// for bit.  kind 0: y[e] = v; 1: d[e] = rope(v, partner e ^ 1) with (cos, sin) cs[(e % ne0) / 2] (and
// y[e] = v unless d is y), then the copy of d[e]; 2: y[e] = v, then the copy of v.  The copy writes
// linear element e of its target view (ne10, ne11, strides in bytes) as F16 or F32 when c != nullptr.
//   glu != 0 instead (two matrices of M rows, gate then up, launched as 2M interleaved rows): the silu -> mul
// that follows w1 | w3, d[0][e] = silu(gate[e]) and d[1][e] = d[0][e] * up[e] as k_silu_mul computes them
// (table: table_silu_f16 as the kernels take it), beside the two outputs
struct GemvEpi {
    int glu;
    const uint16_t *table;
    float *d[GEMV_MULTI_MAX];
    const float2 *cs[GEMV_MULTI_MAX];
    char *c[GEMV_MULTI_MAX];
    int kind[GEMV_MULTI_MAX], f16[GEMV_MULTI_MAX], ne0[GEMV_MULTI_MAX];
    int ne10[GEMV_MULTI_MAX], ne11[GEMV_MULTI_MAX], nb10[GEMV_MULTI_MAX], nb11[GEMV_MULTI_MAX], nb12[GEMV_MULTI_MAX];
};
// epi: nullptr, or the epilogue of every matrix (strided row mapping; returns hipErrorInvalidValue where the
// launch shape cannot pair rows e and e ^ 1 inside one workgroup)
hipError_t gemv_q4_0_multi_norm(int nmat, const void *const *W, const int64_t *M, int64_t K, const float *b,
                                const GemvNorm &nrm, float *const *y, const int64_t *ldy, const DeviceInfo &dev,
                                hipStream_t s, const GemvEpi *epi = nullptr);

// test hook: force the GEMV launch policy (row mapping 0/1/2, ring depth 1/2, row items 0/1,
// workgroups per CU); -1 / 0 = automatic
void gemv_set_policy(int map, int depth, int rowitems, int wg_per_cu);
void gemv_set_bal(int bal);   // -1 auto, 0 off, 1 every chunked decode launch (K > 12288)


// Prefill path: int8 MFMA (v_mfma_i32_32x32x32_i8, K=32 = one q4_0 block) GEMM on the
// pre-quantized activations xs (quantize_q8_0_soa).
// xd16: the same d_x as fp16 bits, block-major [K/32][N] (quantize_q8_0_soa's d16 copy; the default
// LDS GEMM DMAs it straight into its operand layout)
hipError_t gemm_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd,
                     int64_t N, float *y, int64_t ldy, hipStream_t s, const uint16_t *xd16);

// Prefill GEMM v8 (default for the LDS GEMM path): x as a block-major int8 image + fp16 d_x
// (gemm8_prep_x, bit-exact q8_0 values), the q4_0 weights converted per call into an int8 image
// (w = nibble - 8, fp16 d verbatim) in the workspace wws, then the MFMA GEMM over both images.
int64_t gemm8_np(int64_t N);
size_t gemm8_x_bytes(int64_t K, int64_t N);       // x image + d_x
size_t gemm8_w_bytes(int64_t K, int64_t M);       // weight image + d_w
hipError_t gemm8_prep_x(const float *x, int64_t K, int64_t N, void *xws, hipStream_t s);
hipError_t gemm8_prep_w(const void *W, int64_t K, int64_t M, void *wws, hipStream_t s);
hipError_t gemm8_run(const void *wws, int64_t K, int64_t M, const void *xws, int64_t N, float *y, int64_t ldy,
                     hipStream_t s);
// Prefill GEMM v9: the same block sums on the block-scaled fp6 MFMA (e2m3 images: weights w/2,
// x split into (q >> 4)/2 and (q & 15)/2; 26 B per 32 weights, 50 B per 32 activations), bitwise
// equal to v8.
int64_t gemm9_np(int64_t N);
size_t gemm9_x_bytes(int64_t K, int64_t N);
size_t gemm9_w_bytes(int64_t K, int64_t M);
hipError_t gemm9_prep_x(const float *x, int64_t K, int64_t N, void *xws, hipStream_t s);
hipError_t gemm9_prep_w(const void *W, int64_t K, int64_t M, void *wws, hipStream_t s);
// one launch over the row tiles of n (1..4) sibling weight images that share the x image; xo (optional, per
// matrix, null entries allowed): the epilogue also writes matrix i's y as the x image of a next launch (K = M[i],
// same N; bitwise gemm9_prep_x of y; gemm9_xo_ok(M[i], N), ldy[i] == M[i], gemm9_x_bytes(M[i], N) bytes)
bool gemm9_xo_ok(int64_t M, int64_t N);
hipError_t gemm9_run_multi(int n, const void *const *wws, const int64_t *M, int64_t K, const void *xws, int64_t N,
                           float *const *y, const int64_t *ldy, hipStream_t s, uint8_t *const *xo = nullptr);
hipError_t gemm9_run(const void *wws, int64_t K, int64_t M, const void *xws, int64_t N, float *y, int64_t ldy,
                     hipStream_t s);
// the 128 x 128 tile (k_gemm9w): -1 auto by rounds of CUs (GGML_HIP_GEMM9_WIDE overrides), 0 never, 1 always
void gemm9_set_wide(int mode);

// Small / medium N (split-K over the waves of a 32x32-tile workgroup, operands straight to registers).
hipError_t gemm_sk_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                        float *y, int64_t ldy, int num_cus, hipStream_t s);

// Exact mode: y bit-identical to the reference's AVX2+FMA ggml_vec_dot_q4_0_q8_0 (ggml.c:2412-2435),
// per-lane sequential fma chains in block order; any N.
hipError_t mm_exact_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                         float *y, int64_t ldy, hipStream_t s);
// the same for up to 4 matrices of the same K sharing x, one launch (sibling groups in exact mode)
hipError_t mm_exact_q4_0_multi(int n, const void *const *W, const int64_t *M, int64_t K, const int8_t *xqs,
                               const float *xd, int64_t N, float *const *y, const int64_t *ldy, hipStream_t s);

// Multi-GPU helper: y[n*ldy + row0[r] + i] = slab[r][n][i] for i < rows[r] (gather compaction).
// row_begin travels as a kernel argument (no host->device copy, capture-safe)
static constexpr int SCATTER_MAX_RANKS = 256;
struct RowBegins {
    int64_t v[SCATTER_MAX_RANKS + 1];
};
hipError_t scatter_slabs(const float *slabs, int nranks, int64_t max_rows, const RowBegins &row_begin,
                         int64_t N, float *y, int64_t ldy, hipStream_t s);

// Direct-store all-gather over xGMI (p2p_gather.hip): land[r] = rank r's landing buffer as mapped in
// this process ([2 slots][R][cap] floats), flag[r] = its R flag words, ctl = this rank's control block
// (epoch, arrivals, error bits).
constexpr int P2P_MAX_RANKS = 8;
struct P2PArgs {
    float *land[P2P_MAX_RANKS];
    uint64_t *flag[P2P_MAX_RANKS];
    uint64_t *ctl;                   // [0] epoch, [1] arrivals, [2] error bits (peer q timed out: bit q),
                                     // [3] failure notices from peers (peer p failed: bit p, stored by p)
    uint64_t *pctl[P2P_MAX_RANKS];   // every rank's control block (ctl of rank r, mapped here)
    uint32_t *herr;                  // host-mapped words, or nullptr: [0] error (nonzero: the comm failed),
                                     // [1] abort request (set by the host in ggml_hip_comm_abort; polled by
                                     // this rank's own waits, so an in-flight gather ends at its next poll)
    uint64_t timeout;                // peer-wait bound in s_memrealtime ticks (100 MHz)
    int me, R;
    int64_t cap;
};
hipError_t p2p_allgather(const P2PArgs &a, const float *send, int64_t count, float *recv, hipStream_t s);
// fail this rank's comm and notify every peer (bit me in each peer's ctl[3]); stream-ordered on s (the host
// sets herr[1] first, so a gather of this rank blocked ahead of it on s ends and sends the notice itself)
hipError_t p2p_abort(const P2PArgs &a, hipStream_t s);

// Synthetic inputs for the bench (splitmix64 + Box-Muller on device).
hipError_t fill_gaussian(float *dst, int64_t n, uint64_t seed, float mean, float std, hipStream_t s);

}  // namespace ghip
