// q4_0_exact.hip — exact mode: the reference AVX2+FMA fp32 schedule of ggml_vec_dot_q4_0_q8_0, bit for bit.
// Shared device helpers and the HBM layouts: q4_0_device.h / q4_0_kernels.h.
#include "q4_0_device.h"

#include <atomic>

namespace ghip {

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
// three workgroups per CU instead of two (tools/r2_exs.sh: exact decode 467 -> 532 tok/s; 4 slots 377)
constexpr int ex_slots(int nc) { return nc == 1 ? 2 : 3; }

// EXC = blocks per chunk.  64: the weights of a chunk are 18 1-KiB DMAs, 9 per wave, and wave w loads
// half w of each x column.  32 (N = 1 only): 9 weight DMAs, 5 for wave 0 and 4 for wave 1, which loads
// the 1-KiB x column instead, so both waves still issue the same count (6 with the d_x DMA) and half
// the LDS per slot lets twice the workgroups share a CU (tools/r3_exact_c.sh, 2 interleaved rounds: 32 x 2
// slots 549-551 tok/s, 64 x 2 530-533, 32 x 3 518-520)
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
    static std::atomic<uint32_t> attr{0};            // one bit per device (16 max), thread-safe
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev > 15) dev = 0;
    if (!(attr.load(std::memory_order_acquire) & (1u << dev))) {
        hipError_t e = hipFuncSetAttribute((const void *)k_mm_exact_q4_0<NC, EXC, SLOTS>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        attr.fetch_or(1u << dev, std::memory_order_acq_rel);
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
    // columns per workgroup (tools/exact_nc.sh, 4096 x 4096): 8 columns best at N = 8, 2 at N = 40 and 512
    const int nc = N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : 2;
    if (nc == 1) return launch_exact<1, 32>(m, n, K, xqs, xd, N, s);   // decode: 32-block chunks
    if (nc == 2) return launch_exact<2>(m, n, K, xqs, xd, N, s);
    if (nc == 4) return launch_exact<4>(m, n, K, xqs, xd, N, s);
    return launch_exact<8>(m, n, K, xqs, xd, N, s);
}

hipError_t mm_exact_q4_0(const void *W, int64_t K, int64_t M, const int8_t *xqs, const float *xd, int64_t N,
                         float *y, int64_t ldy, hipStream_t s) {
    return mm_exact_q4_0_multi(1, &W, &M, K, xqs, xd, N, &y, &ldy, s);
}

}  // namespace ghip
