// q4_0_gemm.hip — the prefill GEMMs on the matrix cores: k_gemm7 (q4_0 bytes in place), k_gemm8 / k_gemm9
// (int8 / fp6 weight images), and the split-K GEMM for 9 <= N <= 128.
// Shared device helpers and the HBM layouts: q4_0_device.h / q4_0_kernels.h.
#include "q4_0_device.h"

#include <atomic>

namespace {
constexpr int G9_MAX_DEV = 16;
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), thread-safe: a bit per kernel key
// in a per-device atomic mask (the flags were plain function-static bools, set from whichever
// device was current on the first call)
hipError_t lds_attr_once(int key, const void *fn, int bytes) {
    static std::atomic<uint32_t> done[G9_MAX_DEV];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= G9_MAX_DEV) dev = 0;
    if (done[dev].load(std::memory_order_acquire) & (1u << key)) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done[dev].fetch_or(1u << key, std::memory_order_acq_rel);
    return e;
}
}  // namespace

namespace ghip {

// ---------------------------------------------------------------------------------------------
// GEMM (prefill): the LDS GEMMs share one layout vocabulary.  MFMA roles: A = activations (token =
// MFMA row), B = weights (weight row = MFMA column): lane (c, h) = (lane&31, lane>>5) supplies k-half
// h (elements 16h..16h+15) of token c (A) and of weight row c (B).  D[token][row] has the weight row
// on the lane, so each output register is a 128-byte contiguous store and d_w is one value per lane.
// The integer (or fp6-exact) MFMA result is the exact block sum; the epilogue applies d_x[token] *
// d_w[row] in fp32 (one fmaf per output and block).  LDS rows of 32 B have their two 16-byte halves
// swapped when (r>>3)&1, so the ds_read_b128 of 32 consecutive rows hits 16 distinct bank slots.

static constexpr int GM_BM = 64, GM_BN = 128, GM_KB = 4, GM_WAVES = 8, GM_THREADS = GM_WAVES * 64;

__device__ __forceinline__ uint32_t nib_to_i8x4(uint32_t q, int shift) {
    const uint32_t n = (q >> shift) & 0x0F0F0F0Fu;                 // 0..15 per byte
    return ((n | 0x80808080u) - 0x08080808u) ^ 0x80808080u;      // n - 8 as int8, no cross-byte borrow
}

__device__ __forceinline__ int gm_half_off(int r, int half) {    // byte offset of a 16-B half in a 32-B row
    return r * 32 + 16 * (half ^ ((r >> 3) & 1));
}

// ---------------------------------------------------------------------------------------------
// Shared by k_gemm7 (and, through scale_rank1, k_gemm8/9 and split-K): the per-block scale
// d_x[token] * d_w[row] is an exact rank-1 product of two fp16 values, so one fp16 MFMA with d_x at
// k = 0 of A and d_w at k = 0 of B produces all 16 products of a lane in the int8 tile's D layout
// (fp16 x fp16 is exact in fp32: the same value as the CPU's fp32(d_x) * fp32(d_w)).  (The round-2
// v5 / v6 LDS GEMMs that preceded k_gemm7 are in the git history, not in the library.)
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
struct G6Ops {                                                   // one block's MFMA operands
    i32x4 a, b;
    uint32_t sx, sw;
};

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
        const __amdgpu_buffer_rsrc_t wr_ = valid ? wrs : nul;
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

// Schedule (round 3, tools/r3_g8var.sh, kernel medians at 4096x4096x512: 33.3 -> 29.2 us): the i8
// MFMA accumulates on 0 and the epilogue converts with v_cvt_f32_i32 (no 16-register bias operand to
// keep live or rebuild); the next block's operands are read from LDS while the current block
// computes; each block's four MFMAs issue back to back and both epilogues follow.  (The A/B variants
// and timing knockouts of that measurement are in the git history.)
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
        if (wave < 8) return;
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
    const i32x16 im = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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
            a[i] = fmaf((float)S[i], P[i], a[i]);
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
    };
    auto sync = [&]() __attribute__((always_inline)) {   // retire stage s+1, keep s+2 in flight
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((G8_NS - 2) * G8_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    };

    const int nstages = (nb + G8_KB - 1) / G8_KB;
#pragma unroll
    for (int st = 0; st < G8_NS - 1; st++) issue(st);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((G8_NS - 2) * G8_OPS) : "memory");   // stage 0 landed
    __builtin_amdgcn_s_barrier();
    for (int s = 0; s < nstages; s++) {
        issue(s + G8_NS - 1);
        const int kb = s * G8_KB + 4 * g;
        if (wave < 8) {                            // nb is even and kb too: blocks come in valid pairs
            Ops o = rd(s, 4 * g);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (kb + j >= nb) break;
                Ops n = o;
                if (j < 3) n = rd(s, 4 * g + j + 1);
                block(o);
                o = n;
            }
        }
        sync();
    }
    epi(acc0, S0, P0);
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
    if (const hipError_t e = lds_attr_once(0, (const void *)k_gemm8_q4_0, G8_LDS); e != hipSuccess) return e;
    (void)hipGetLastError();
    launch_k(k_gemm8_q4_0, dim3((unsigned)Mt, (unsigned)((N + G8_BN - 1) / G8_BN)), dim3(G8_THREADS), G8_LDS, s, wimg, wd16,
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

// 32 codes = fields F0..F7 (24 bits each) -> 6 dwords, element j at bits 6j..6j+5
__device__ __forceinline__ void f6_pack(const uint32_t *F, uint32_t *D) {
    D[0] = F[0] | (F[1] << 24);
    D[1] = (F[1] >> 8) | (F[2] << 16);
    D[2] = (F[2] >> 16) | (F[3] << 8);
    D[3] = F[4] | (F[5] << 24);
    D[4] = (F[5] >> 8) | (F[6] << 16);
    D[5] = (F[6] >> 16) | (F[7] << 8);
}

// x: 8 lanes per block (x9_store_lane), wave = 8 tokens of one block.  (Two or four blocks per wave with
// all their loads in flight measured equal or slower: 0.338-0.345 vs 0.338-0.340 ms per prefill layer.)
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
    x9_store_lane(v, sub, n, b, live, ximg, xd16, Np);
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

// Schedule (round 3, each step measured interleaved on one box, tools/r3_g9*.sh; the rejected variants
// are in the git history): operands read right before their block from per-stage VGPR address bases
// with the block offsets as ds_read immediates (no address VALU per block); the second weight tile's
// 8-byte part from its own opaque base (no ds_read2 pairing + v_mov reassembly); the rank-1 scale
// product on the K = 8 fp16 MFMA; each block's MFMA burst ordered fp6, fp6, fp16, fp16, the previous
// block's two epilogues ahead of it.
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
    int nfull;                  // tiles [0, nfull) run whole; each later tile runs as two 64-row halves
    int toff;                   // 128 x 64 launch after a 128 x 128 one: its tiles start at this index (xcd order)
    // prefill chains (ggml_hip_chain_create_n): matrix i's y is the next launch's x, and the epilogue writes that
    // launch's x image from the f32 values it stores (null: no image; M[i] % 64 == 0, image Np = this launch's)
    uint8_t *xo[4];
};

// The epilogue's x image (prefill chains): the workgroup's f32 outputs staged in LDS as [token][row] (row
// stride G9_TS floats), then 8 lanes per (token, 32-row block) run x9_store_lane on them, exactly what
// k_prep9_x does with the same floats read from y: the image is bitwise gemm9_prep_x's of y.  ntok x nrow
// is the workgroup's tile (rows from its first, m0 = the tile's first row of the matrix); every thread of
// the workgroup calls it, BEFORE the tile's y stores: the compiler puts s_waitcnt vmcnt(0) ahead of any LDS
// read while global stores may be in flight (it cannot tell them from the LDS DMAs), so every T read is
// issued first, with nothing outstanding, and the image stores last (+15-20 % per launch the other way round).
static constexpr int G9_TS = 136;                   // 544 B: 16-byte aligned rows, tokens 4 apart on other banks
// a workgroup barrier for LDS only (__syncthreads() also waits for outstanding global memory operations);
// the asm clobbers keep the compiler's LDS accesses on their side of it
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
template <int NTOK, int NROW>
__device__ __forceinline__ void g9_ximage_out(const float *T, int m0, int n0, int M, int N, int nbo, uint8_t *xo,
                                              int64_t Np) {
    constexpr int ITEMS = NTOK * (NROW / 32), PER = G9_THREADS / 8, IT = (ITEMS + PER - 1) / PER;
    uint16_t *xod = reinterpret_cast<uint16_t *>(xo + (int64_t)nbo * Np * 48);
    const int sub = threadIdx.x & 7;
    float4 v[IT];
    bool live[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const int it = k * PER + (int)(threadIdx.x >> 3);
        const int blk = it / NTOK, tok = it - blk * NTOK;
        live[k] = it < ITEMS && n0 + tok < N && m0 + 32 * blk + 32 <= M;
        v[k] = live[k] ? *reinterpret_cast<const float4 *>(T + tok * G9_TS + 32 * blk + 4 * sub) : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {                          // every lane calls x9_store_lane (DPP)
        const int it = k * PER + (int)(threadIdx.x >> 3);
        const int blk = it / NTOK, tok = it - blk * NTOK;
        x9_store_lane(v[k], sub, n0 + tok, (m0 >> 5) + blk, live[k], xo, xod, Np);
    }
}

// Timing-only diagnostic builds (tools/build_variant.sh FILE=q4_0_gemm -DGEMM9_KO=n; results invalid):
// 1 = no LDS DMAs at all (compute only), 2 = no x code DMAs, 3 = no weight code DMAs.
#ifndef GEMM9_KO
#define GEMM9_KO 0
#endif

// HALF: the workgroup computes rows [64 hsel, 64 hsel + 64) of its 128-row tile, one 32 x 32 tile per compute
// wave (the same per-output arithmetic: bitwise the whole tile's values for those rows).  Tile order: see
// G9Mats; the HALF instantiation runs the tiles from mats.nfull on, two workgroups per tile (gemm9_run_multi:
// the last partial round of a multi-round launch, e.g. LLaMA-7B w1|w3 at N = 512 = 5 rounds of 256 + 96).
// (One kernel with both forms behind a workgroup-uniform branch spilled 200 bytes: two instantiations.)
template <bool HALF>
__global__ __launch_bounds__(G9_THREADS, 1) void k_gemm9_q4_0(const G9Mats mats, int nb,
                                                               const uint8_t *__restrict__ ximg,
                                                               const uint16_t *__restrict__ xd16, int64_t Np, int N) {
    const int Mt = mats.tb[mats.n];
    int j = (int)blockIdx.x, hsel = 0;
    if constexpr (HALF) {
        hsel = j & 1;
        j = mats.nfull + (j >> 1);
    } else if (mats.xcd) {
        const int C = (int)gridDim.x >> 3;
        if (j < 8 * C) j = (j & 7) * C + (j >> 3);
    }
    j += mats.toff;
    const int rtg = mats.xcd ? j / mats.ny : j % Mt, ty = mats.xcd ? j - rtg * mats.ny : j / Mt;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *zero = smem + G9_NS * G9_STAGE;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
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
        if (wave < 8 || GEMM9_KO == 1) return;
        uint8_t *base = smem + (st % G9_NS) * G9_STAGE;
        const int kb0 = st * G9_KB;
        const bool v = kb0 + lb < nb;                                             // nb even: both or none
        const __amdgpu_buffer_rsrc_t wr_ = v ? wrs : nul, xr_ = v ? xrs : nul, dr_ = v ? xdrs : nul,
                                     wdr_ = v ? wdrs : nul;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int b = lb + j;
#pragma unroll
            for (int r = 0; r < 3; r++)
                if (GEMM9_KO != 3)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr_, (lds_void_t *)(base + b * G9_WB + r * 1024), 16,
                                                         (kb0 + b) * G9_WB + r * 1024 + lane * 16, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 3; r++)
                if (GEMM9_KO != 2)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_, (lds_void_t *)(base + G9_W + b * G9_XB + r * 1024), 16,
                                                         (int)((((int64_t)(kb0 + b) * 3 + r) * Np + n0) * 16) + lane * 16,
                                                         0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wdr_, (lds_void_t *)(base + G9_W + G9_X + b * 256), 4,
                                                     (kb0 + b) * 256 + lane * 4, 0, 0, 0);
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dr_, (lds_void_t *)(base + G9_W + G9_X + G9_WD + lb * 128), 4,
                                                 (int)(((int64_t)(kb0 + lb + h) * Np + n0) * 2) + c * 4, 0, 0, 0);
    };
    const int g = (wave >> 2) & 1, q = wave & 3;
    const int tt = 32 * (q & 1) + c;                       // this lane's token (A operand row) in the tile
    const int r0 = HALF ? 64 * hsel + 32 * (q >> 1) + c : 64 * (q >> 1) + c;   // this lane's weight rows
    const int r1 = r0 + 32;                                                   // (B operand columns)
    const int xo16 = h * 1024 + tt * 16, xo8 = 2048 + tt * 16 + 8 * (h ^ ((tt >> 4) & 1));
    const int sa = h ? G9_SCALE_1 : G9_SCALE_5;
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float acc0[16], acc1[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.0f;
    f32x16 S0 = fz, S1 = fz, P0 = fz, P1 = fz;
    u32x4 as = {0u, 0u, 0u, 0u}, bs0 = {0u, 0u, 0u, 0u}, bs1 = {0u, 0u, 0u, 0u};
    auto epi = [&](float *a, const f32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; i++) a[i] = fmaf(S[i], P[i], a[i]);
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
    auto block = [&](const Ops &o) __attribute__((always_inline)) {
        as.x = o.sx;
        bs0.x = o.sw0;
        bs1.x = o.sw1;
        // the previous block's epilogues, then this block's four MFMAs back to back: the two fp6 MFMAs,
        // then the two fp16 ones (two format switches per burst, not four)
        epi(acc0, S0, P0);
        if constexpr (!HALF) epi(acc1, S1, P1);
        __builtin_amdgcn_sched_barrier(0);
        S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw0, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
        if constexpr (!HALF) S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw1, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
        P0 = scale_rank1(as, bs0);
        if constexpr (!HALF) P1 = scale_rank1(as, bs1);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((G9_NS - 2) * G9_OPS) : "memory");
        __builtin_amdgcn_s_barrier();
    };

    const int nstages = (nb + G9_KB - 1) / G9_KB;
#pragma unroll
    for (int st = 0; st < G9_NS - 1; st++) issue(st);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((G9_NS - 2) * G9_OPS) : "memory");
    __builtin_amdgcn_s_barrier();
    for (int s = 0; s < nstages; s++) {
        issue(s + G9_NS - 1);
        const int kb = s * G9_KB + 4 * g;
        if (wave < 8) {
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
                if constexpr (HALF) o.bw1 = o.bw0;
                else o.bw1 = rd24(smem + wa1 + j * G9_WB, smem + w81 + j * G9_WB);
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
        }
        sync();
    }
    epi(acc0, S0, P0);
    if constexpr (!HALF) epi(acc1, S1, P1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float *red = reinterpret_cast<float *>(smem);
    if (wave >= 4 && wave < 8) {
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            *reinterpret_cast<float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4) = {acc0[i], acc0[i + 1], acc0[i + 2], acc0[i + 3]};
            if constexpr (!HALF)
                *reinterpret_cast<float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4) = {acc1[i], acc1[i + 1], acc1[i + 2], acc1[i + 3]};
        }
    }
    __syncthreads();
    uint8_t *xo = mi == 0 ? mats.xo[0] : mi == 1 ? mats.xo[1] : mi == 2 ? mats.xo[2] : mats.xo[3];
    float *T = red + 8 * 256 * 4;                               // the epilogue's stage, after red (32 KB)
    if (wave < 4) {
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            const float4 o0 = *reinterpret_cast<const float4 *>(red + ((i / 4) * 256 + q * 64 + lane) * 4);
            acc0[i] += o0.x; acc0[i + 1] += o0.y; acc0[i + 2] += o0.z; acc0[i + 3] += o0.w;
            if constexpr (!HALF) {
                const float4 o1 = *reinterpret_cast<const float4 *>(red + ((4 + i / 4) * 256 + q * 64 + lane) * 4);
                acc1[i] += o1.x; acc1[i + 1] += o1.y; acc1[i + 2] += o1.z; acc1[i + 3] += o1.w;
            }
        }
        if (xo) {
            const int l0 = r0 - (HALF ? 64 * hsel : 0);         // the row within this workgroup's rows
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int tl = 32 * (q & 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
                T[tl * G9_TS + l0] = acc0[i];
                if constexpr (!HALF) T[tl * G9_TS + l0 + 32] = acc1[i];
            }
        }
    }
    if (xo) {                                                   // workgroup-uniform
        lds_barrier();
        g9_ximage_out<G9_BN, HALF ? 64 : G9_BM>(T, m0 + (HALF ? 64 * hsel : 0), n0, M, N, M >> 5, xo, Np);
    }
    if (wave < 4) {
        const int row0 = m0 + r0, row1 = m0 + r1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int tk = n0 + 32 * (q & 1) + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (tk < N) {
                if (row0 < M) y[(int64_t)tk * ldy + row0] = acc0[i];
                if (!HALF && row1 < M) y[(int64_t)tk * ldy + row1] = acc1[i];
            }
        }
    }
}

// The larger tile (round 5, verdict r4 item 3): 128 rows x 128 tokens per workgroup, half the LDS-DMA bytes
// of x per MFMA (a block stage moves 3 KB of weight codes + 6 KB of x codes for 16 tile MFMAs instead of
// 3 + 3 KB for 8).  No K split between waves: compute wave w owns tokens 32 (w & 3) .. and rows
// 64 (w >> 2) + {0, 32} over every block of a stage (k_gemm9's two-tile operand reuse); stage 76 KB, ring
// of 2.  The same per-block integer sums and scale products as k_gemm9, summed in block order (k_gemm9 sums
// blocks 0-3 and 4-7 of every stage apart and adds the two at the end; keeping both partial sums here needs
// 32 more VGPRs than the 168 a wave has at 3 waves per SIMD: 279 spilled): y is within the oracle bound of
// k_gemm9's, not bitwise, so gemm9_run_multi's choice is a function of the launch's tile counts and the
// tests pin the mode wherever they compare two launches bitwise.  gemm9_run_multi picks it per launch by
// rounds of CUs (wide_pays).  Knockouts as GEMM9_KO.
static constexpr int W9_BN = 128, W9_NS = 2;
static constexpr int W9_XB = W9_BN * 48;                          // 6 KB
static constexpr int W9_X = G9_KB * W9_XB;                        // 48 KB
static constexpr int W9_XD = G9_KB * W9_BN * 2;                   // 2 KB
static constexpr int W9_STAGE = G9_W + W9_X + G9_WD + W9_XD;      // 76 KB
static constexpr int W9_ZERO = 2048;                                // zero d_w: 8 blocks x 256 B
static constexpr int W9_LDS = W9_NS * W9_STAGE + W9_ZERO;          // 154 KB

__global__ __launch_bounds__(G9_THREADS, 1) void k_gemm9w_q4_0(const G9Mats mats, int nb,
                                                                const uint8_t *__restrict__ ximg,
                                                                const uint16_t *__restrict__ xd16, int64_t Np, int N) {
    const int Mt = mats.tb[mats.n];
    int j = (int)blockIdx.x;
    if (mats.xcd) {
        const int C = (int)gridDim.x >> 3;
        if (j < 8 * C) j = (j & 7) * C + (j >> 3);
    }
    const int rtg = mats.xcd ? j / mats.ny : j % Mt, ty = mats.xcd ? j - rtg * mats.ny : j / Mt;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *zero = smem + W9_NS * W9_STAGE;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 31, h = lane >> 5;
    const int mi = (mats.n > 1 && rtg >= mats.tb[1]) + (mats.n > 2 && rtg >= mats.tb[2]) + (mats.n > 3 && rtg >= mats.tb[3]);
    const uint8_t *wimg = mi == 0 ? mats.wimg[0] : mi == 1 ? mats.wimg[1] : mi == 2 ? mats.wimg[2] : mats.wimg[3];
    const uint16_t *wd16 = mi == 0 ? mats.wd16[0] : mi == 1 ? mats.wd16[1] : mi == 2 ? mats.wd16[2] : mats.wd16[3];
    float *y = mi == 0 ? mats.y[0] : mi == 1 ? mats.y[1] : mi == 2 ? mats.y[2] : mats.y[3];
    const int64_t ldy = mi == 0 ? mats.ldy[0] : mi == 1 ? mats.ldy[1] : mi == 2 ? mats.ldy[2] : mats.ldy[3];
    const int M = mi == 0 ? mats.M[0] : mi == 1 ? mats.M[1] : mi == 2 ? mats.M[2] : mats.M[3];
    const int rt = rtg - (mi == 0 ? 0 : mi == 1 ? mats.tb[1] : mi == 2 ? mats.tb[2] : mats.tb[3]);
    const int m0 = rt * G9_BM, n0 = ty * W9_BN;
    if (tid < W9_ZERO / 4) reinterpret_cast<uint32_t *>(zero)[tid] = 0u;

    const __amdgpu_buffer_rsrc_t wrs = make_rsrc(wimg + (int64_t)rt * nb * G9_WB, (uint32_t)nb * G9_WB);
    const __amdgpu_buffer_rsrc_t wdrs = make_rsrc(wd16 + (int64_t)rt * nb * G9_BM, (uint32_t)nb * G9_BM * 2u);
    const __amdgpu_buffer_rsrc_t xrs = make_rsrc(ximg, (uint32_t)((int64_t)nb * Np * 48));
    const __amdgpu_buffer_rsrc_t xdrs = make_rsrc(xd16, (uint32_t)((int64_t)nb * Np * 2));
    const __amdgpu_buffer_rsrc_t nul = make_rsrc(wimg, 0);

    const int lb = 2 * (wave - 8);
    auto issue = [&](int st) __attribute__((always_inline)) {
        if (wave < 8 || GEMM9_KO == 1) return;
        uint8_t *base = smem + (st % W9_NS) * W9_STAGE;
        const int kb0 = st * G9_KB;
        const bool v = kb0 + lb < nb;
        const __amdgpu_buffer_rsrc_t wr_ = v ? wrs : nul, xr_ = v ? xrs : nul, dr_ = v ? xdrs : nul,
                                     wdr_ = v ? wdrs : nul;
#pragma unroll
        for (int jj = 0; jj < 2; jj++) {
            const int b = lb + jj;
#pragma unroll
            for (int r = 0; r < 3; r++)
                if (GEMM9_KO != 3)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr_, (lds_void_t *)(base + b * G9_WB + r * 1024), 16,
                                                         (kb0 + b) * G9_WB + r * 1024 + lane * 16, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int hh = 0; hh < 2; hh++)
                    if (GEMM9_KO != 2)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        xr_, (lds_void_t *)(base + G9_W + b * W9_XB + r * 2048 + hh * 1024), 16,
                        (int)((((int64_t)(kb0 + b) * 3 + r) * Np + n0 + 64 * hh) * 16) + lane * 16, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wdr_, (lds_void_t *)(base + G9_W + W9_X + b * 256), 4,
                                                     (kb0 + b) * 256 + lane * 4, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dr_, (lds_void_t *)(base + G9_W + W9_X + G9_WD + b * 256), 4,
                                                     (int)(((int64_t)(kb0 + b) * Np + n0) * 2) + lane * 4, 0, 0, 0);
        }
    };
    const int tq = wave & 3, rh = (wave >> 2) & 1;
    const int tt = 32 * tq + c;
    const int r0 = 64 * rh + c, r1 = r0 + 32;
    const int xo16 = h * 2048 + tt * 16, xo8 = 4096 + tt * 16 + 8 * (h ^ ((tt >> 4) & 1));
    const int sa = h ? G9_SCALE_1 : G9_SCALE_5;
    const f32x16 fz = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    float acc0[16], acc1[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc0[i] = acc1[i] = 0.0f;
    f32x16 S0 = fz, S1 = fz, P0 = fz, P1 = fz;
    u32x4 as = {0u, 0u, 0u, 0u}, bs0 = {0u, 0u, 0u, 0u}, bs1 = {0u, 0u, 0u, 0u};
    auto epi = [&](float *a, const f32x16 &S, const f32x16 &P) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 16; i++) a[i] = fmaf(S[i], P[i], a[i]);
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
    auto block = [&](const Ops &o) __attribute__((always_inline)) {
        as.x = o.sx;
        bs0.x = o.sw0;
        bs1.x = o.sw1;
        epi(acc0, S0, P0);
        epi(acc1, S1, P1);
        __builtin_amdgcn_sched_barrier(0);
        S0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw0, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
        S1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(o.ax, o.bw1, fz, 2, 2, 0, sa, 0, G9_SCALE_1);
        P0 = scale_rank1(as, bs0);
        P1 = scale_rank1(as, bs1);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto sync = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    const int nstages = (nb + G9_KB - 1) / G9_KB;
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int s = 0; s < nstages; s++) {
        issue(s + 1);
        const int kb = s * G9_KB;
        if (wave < 8) {
            const uint32_t sb = (uint32_t)(s % W9_NS) * W9_STAGE;
            uint32_t xa = sb + G9_W + xo16, xb8 = sb + G9_W + xo8;
            uint32_t wa0 = sb + r0 * 16, wa1 = wa0 + 512;
            uint32_t w80 = sb + 2048 + r0 * 8, w81 = w80 + 256;
            uint32_t da = h ? (uint32_t)(W9_NS * W9_STAGE) : sb + G9_W + W9_X + r0 * 2;
            uint32_t xd = sb + G9_W + W9_X + G9_WD + tt * 2;
            asm volatile("" : "+v"(wa1), "+v"(w81));
            auto rdj = [&](int jb) __attribute__((always_inline)) {
                Ops o;
                o.ax = rd24(smem + xa + jb * W9_XB, smem + xb8 + jb * W9_XB);
                o.bw0 = rd24(smem + wa0 + jb * G9_WB, smem + w80 + jb * G9_WB);
                o.bw1 = rd24(smem + wa1 + jb * G9_WB, smem + w81 + jb * G9_WB);
                o.sw0 = *reinterpret_cast<const uint16_t *>(smem + da + jb * 256);
                o.sw1 = *reinterpret_cast<const uint16_t *>(smem + da + jb * 256 + 64);
                o.sx = *reinterpret_cast<const uint16_t *>(smem + xd + jb * 256);
                return o;
            };
#pragma unroll
            for (int jb = 0; jb < G9_KB; jb++) {
                if (kb + jb >= nb) break;
                block(rdj(jb));
            }
        }
        sync();
    }
    epi(acc0, S0, P0);
    epi(acc1, S1, P1);
    uint8_t *xo = mi == 0 ? mats.xo[0] : mi == 1 ? mats.xo[1] : mi == 2 ? mats.xo[2] : mats.xo[3];
    if (xo) {                                                   // workgroup-uniform; the last sync drained the DMAs
        float *T = reinterpret_cast<float *>(smem);
        if (wave < 8) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int tl = 32 * tq + (i & 3) + 8 * (i >> 2) + 4 * h;
                T[tl * G9_TS + r0] = acc0[i];
                T[tl * G9_TS + r1] = acc1[i];
            }
        }
        lds_barrier();
        g9_ximage_out<W9_BN, G9_BM>(T, m0, n0, M, N, M >> 5, xo, Np);
    }
    if (wave < 8) {
        const int row0 = m0 + r0, row1 = m0 + r1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int tk = n0 + 32 * tq + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (tk < N) {
                if (row0 < M) y[(int64_t)tk * ldy + row0] = acc0[i];
                if (row1 < M) y[(int64_t)tk * ldy + row1] = acc1[i];
            }
        }
    }
}


// wide tile choice: -1 auto (GGML_HIP_GEMM9_WIDE unset), 0 never, 1 always (tests / A/B)
static std::atomic<int> g_wide_mode{env_int("GGML_HIP_GEMM9_WIDE", -1)};
void gemm9_set_wide(int mode) { g_wide_mode.store(mode < 0 ? env_int("GGML_HIP_GEMM9_WIDE", -1) : mode, std::memory_order_relaxed); }

// Which tile, by rounds of one-workgroup-per-CU tiles (fit to tools/g9_tile_sweep.py over the LLaMA-7B / 13B and
// Falcon-7B prefill launches at 128-2048 tokens, profiles/r05_gemm9_tile_sweep.txt): 128 x 64 when its tiles fit one
// round; else 128 x 128 when its tiles fit one round, fill at least two, or leave a last round more than half full
// (a last 128 x 128 round at most half full costs nearly a full one while 128 x 64 runs its tail as half tiles:
// 1.03-1.18x at 1.1-1.5 rounds).
static bool wide_pays(int64_t tiles, int64_t tiles_w, int cus) {
    if (tiles <= cus) return false;
    if (tiles_w <= cus || tiles_w >= 2 * (int64_t)cus) return true;
    return 2 * (tiles_w - cus) > cus;
}

int64_t gemm9_np(int64_t N) { return (N + 3) & ~(int64_t)3; }
size_t gemm9_x_bytes(int64_t K, int64_t N) { return (size_t)(K / QK) * gemm9_np(N) * 50; }
size_t gemm9_w_bytes(int64_t K, int64_t M) { return (size_t)((M + 127) / 128) * (K / QK) * 128 * 26; }

hipError_t gemm9_prep_x(const float *x, int64_t K, int64_t N, void *xws, hipStream_t s) {
    const int64_t nb = K / QK;
    if (N <= 0 || nb <= 0) return hipSuccess;
    if ((N + 7) / 8 > 65535) return hipErrorInvalidValue;
    const int64_t Np = gemm9_np(N);
    if (!x9_fits(K, Np)) return hipErrorInvalidValue;
    uint8_t *ximg = (uint8_t *)xws;
    uint16_t *xd16 = (uint16_t *)((char *)xws + (size_t)nb * Np * 48);
    (void)hipGetLastError();
    launch_k(k_prep9_x, dim3((unsigned)((nb + 3) / 4), (unsigned)((N + 7) / 8)), dim3(256), 0, s, x, K, N, ximg, xd16, Np);
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

// whether an epilogue can write an M-row output at N tokens as the next launch's x image (the tile epilogue's
// 64-row granules, its 32-bit image offsets)
bool gemm9_xo_ok(int64_t M, int64_t N) {
    const int64_t Np = gemm9_np(N);
    return M > 0 && M % 64 == 0 && N > 0 && x9_fits(M, Np) && (M / QK) * Np * 48 < ((int64_t)1 << 31);
}

hipError_t gemm9_run_multi(int n, const void *const *wws, const int64_t *Mv, int64_t K, const void *xws, int64_t N,
                           float *const *yv, const int64_t *ldyv, hipStream_t s, uint8_t *const *xo) {
    const int nb = (int)(K / QK);
    const int64_t Np = gemm9_np(N), Ny = (N + G9_BN - 1) / G9_BN;
    if (n < 1 || n > 4 || N <= 0 || nb <= 0) return hipErrorInvalidValue;
    G9Mats mats{};
    for (int i = 0; i < n && xo; i++) {
        if (!xo[i]) continue;
        if (ldyv[i] != Mv[i] || !gemm9_xo_ok(Mv[i], N)) return hipErrorInvalidValue;
        mats.xo[i] = xo[i];
    }
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
    // a last partial round of at most half the CUs runs as twice as many 64-row half tiles, each about half
    // a tile's time (one workgroup per CU: 154 KB of LDS), and so does a whole launch of at most half the CUs
    // (10-27 % faster at 96-192 tokens on the wo / w2 shapes, profiles/r05_gemm9_small_halves.txt);
    // GGML_HIP_GEMM9_HALF=1 keeps only the tail, 0 runs every tile whole
    static const int half_on = env_int("GGML_HIP_GEMM9_HALF", 2);
    // the CU count of the device this launch runs on (devices of one process may differ, e.g. partitions)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= G9_MAX_DEV) dev = 0;
    static std::atomic<int> cus_of[G9_MAX_DEV];
    int cus = cus_of[dev].load(std::memory_order_relaxed);
    if (cus <= 0) {
        int v = 0;
        cus = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
        cus_of[dev].store(cus, std::memory_order_relaxed);
    }
    const int64_t rem = tiles % cus;
    const bool halves = (half_on && tiles > cus && rem > 0 && 2 * rem <= cus) || (half_on == 2 && 2 * tiles <= cus);
    mats.nfull = (int)(halves ? tiles - rem : tiles);
    const int64_t grid = halves ? tiles + rem : tiles;
    const uint8_t *ximg = (const uint8_t *)xws;
    const uint16_t *xd16 = (const uint16_t *)((const char *)xws + (size_t)nb * Np * 48);
    if ((int64_t)nb * Np * 48 >= ((int64_t)1 << 31) || (int64_t)nb * G9_WB >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    const int64_t Nyw = (N + W9_BN - 1) / W9_BN, tiles_w = (int64_t)mats.tb[n] * Nyw;
    const int wm = g_wide_mode.load(std::memory_order_relaxed);
    // Mixed (GGML_HIP_GEMM9_MIXED=0 turns it off): a launch whose 128 x 128 tiles would leave a last round at most half
    // full runs its whole rounds of them (row tiles [0, R)) and the remaining row tiles as 128 x 64, that launch's
    // tail as half tiles: 5-10 % below the faster single tile (profiles/r05_gemm9_mixed.txt); rows [0, 128 R) are
    // bitwise the 128 x 128 tile's, the rest the 128 x 64 tile's.
    static const int mixed_on = env_int("GGML_HIP_GEMM9_MIXED", 1);
    const int64_t rem_w = tiles_w % cus, R = Nyw > 0 ? (tiles_w / cus) * cus / Nyw : 0;
    if (mixed_on && wm == -1 && mats.xcd && tiles > cus && tiles_w > cus && rem_w > 0 && 2 * rem_w <= cus && R > 0 &&
        R < mats.tb[n]) {
        hipError_t e = lds_attr_once(1, (const void *)k_gemm9w_q4_0, W9_LDS);
        if (e == hipSuccess) e = lds_attr_once(2, (const void *)k_gemm9_q4_0<false>, G9_LDS);
        if (e == hipSuccess) e = lds_attr_once(3, (const void *)k_gemm9_q4_0<true>, G9_LDS);
        if (e != hipSuccess) return e;
        (void)hipGetLastError();
        G9Mats mw = mats;                               // row tiles [0, R): 128 x 128
        mw.ny = (int)Nyw;
        mw.toff = 0;
        launch_k(k_gemm9w_q4_0, dim3((unsigned)(R * Nyw)), dim3(G9_THREADS), W9_LDS, s, mw, nb, ximg, xd16, Np, (int)N);
        G9Mats mb = mats;                               // row tiles [R, Mt): 128 x 64, tail as half tiles
        const int64_t tb2 = ((int64_t)mats.tb[n] - R) * Ny, rem2 = tb2 % cus;
        const bool halves2 = half_on && rem2 > 0 && 2 * rem2 <= cus;
        mb.toff = (int)(R * Ny);
        mb.nfull = (int)(halves2 ? tb2 - rem2 : tb2);
        const int64_t grid2 = halves2 ? tb2 + rem2 : tb2;
        if (mb.nfull > 0)
            launch_k(k_gemm9_q4_0<false>, dim3((unsigned)mb.nfull), dim3(G9_THREADS), G9_LDS, s, mb, nb, ximg, xd16, Np, (int)N);
        if (grid2 > mb.nfull)
            launch_k(k_gemm9_q4_0<true>, dim3((unsigned)(grid2 - mb.nfull)), dim3(G9_THREADS), G9_LDS, s, mb, nb, ximg, xd16,
                     Np, (int)N);
        return hipGetLastError();
    }
    if (wm == 1 || (wm == -1 && wide_pays(tiles, tiles_w, cus))) {
        if (const hipError_t e = lds_attr_once(1, (const void *)k_gemm9w_q4_0, W9_LDS); e != hipSuccess) return e;
        mats.ny = (int)Nyw;
        (void)hipGetLastError();
        launch_k(k_gemm9w_q4_0, dim3((unsigned)tiles_w), dim3(G9_THREADS), W9_LDS, s, mats, nb, ximg, xd16, Np, (int)N);
        return hipGetLastError();
    }
    {
        hipError_t e = lds_attr_once(2, (const void *)k_gemm9_q4_0<false>, G9_LDS);
        if (e == hipSuccess) e = lds_attr_once(3, (const void *)k_gemm9_q4_0<true>, G9_LDS);
        if (e != hipSuccess) return e;
    }
    (void)hipGetLastError();
    if (mats.nfull > 0)
        launch_k(k_gemm9_q4_0<false>, dim3((unsigned)mats.nfull), dim3(G9_THREADS), G9_LDS, s, mats, nb, ximg, xd16, Np, (int)N);
    if (grid > mats.nfull)
        launch_k(k_gemm9_q4_0<true>, dim3((unsigned)(grid - mats.nfull)), dim3(G9_THREADS), G9_LDS, s, mats, nb, ximg, xd16,
                 Np, (int)N);
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
    // 16 waves split K while the tiles cover fewer than two rounds of the CUs, 8 above; ring depth 2
    const int sk = tiles < 2 * (int64_t)num_cus ? 16 : 8;
    (void)hipGetLastError();  // report only this launch's error
    if (sk == 16)
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
    if (const hipError_t e = lds_attr_once(4, (const void *)k_gemm7_q4_0, G7_LDS); e != hipSuccess) return e;
    (void)hipGetLastError();  // report only this launch's error
    if (!xd16) return hipErrorInvalidValue;
    launch_k(k_gemm7_q4_0, grid, dim3(GM_THREADS), G7_LDS, s, (const uint8_t *)W, rowbytes, nb, (int)M, xqs, xd16,
             (int)N, (int)K, y, ldy);
    return hipGetLastError();
}

}  // namespace ghip
