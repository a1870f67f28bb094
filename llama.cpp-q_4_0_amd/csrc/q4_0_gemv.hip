// q4_0_gemv.hip — the decode GEMV (N <= 8): q8_0 of x fused into the prologue + q4_0.q8_0 row dots.
// Shared device helpers and the HBM layouts: q4_0_device.h / q4_0_kernels.h.
#include "q4_0_device.h"

namespace ghip {

// ---------------------------------------------------------------------------------------------
// GEMV (decode, N <= 8).
//
// Lane p of a wave owns block pair p of a weight row (and p+64, p+128, ... with row items).  A
// pair is 36 bytes (9 dwords): the 18-byte blocks of a row start 4-byte aligned every second
// block, so a pair is always dword aligned and the 64 lanes of one load read 2,304 contiguous
// bytes (a whole K=4096 row).  Loads are global_load_dwordx4/x4/x1 with clamped lane addresses.  The
// even block's qs are re-aligned with v_alignbyte_b32.  x is quantized once per workgroup into
// LDS (q8_0 ints + fp32 d + 8*sum(q)); the q4_0 nibbles enter v_dot4c_i32_i8 unsigned (0..15)
// and the -8 offset is applied once per block as -8*sum(q):  sum((n-8)*q) = sum(n*q) - 8*sum(q).
//
// Schedule: the x-waves load + quantize x while every other wave already streams its first
// DEPTH items; after the barrier each wave walks its items (whole rows with PPL > 0, 64-pair
// chunks otherwise) with DEPTH items in flight.  Launch policy (grid, row mapping, depth, row
// items) in launch_gemv_w / launch_gemv; every policy gives bitwise-identical results.

static constexpr int GEMV_LDS_MAX = 64 * 1024;
static constexpr int GEMV_XPRO = 4;
#ifndef GEMV_XPRO_N
#define GEMV_XPRO_N 2       // the same for the norm prologue (PRO 1): x-waves = K / (256 * GEMV_XPRO_N); 2: 8 x-waves at
                            // K = 4096 (profiles/r05_gemv_norm_xwaves_ab.txt: q|k|v 0.3 us faster than 4)
#endif         // x float4 loads in flight per x-wave thread in the prologue
static constexpr int GEMV_WAVES = 16;       // waves per workgroup
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
// a / b for a < 2^20, 1 <= b < 2^20 (the epilogue's element indices): a float reciprocal estimate and
// one correction (the estimate is within 1 of the quotient there)
__device__ __forceinline__ uint32_t udiv20(uint32_t a, uint32_t b) {
    int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
    const int rem = (int)a - q * (int)b;
    q += rem < 0 ? -1 : (rem >= (int)b ? 1 : 0);
    return (uint32_t)q;
}
struct GemvTailEpi : GemvTail {
    GemvEpi epi;                          // EPI instantiations (q4_0_kernels.h)
};
template <int EPI> struct GemvTailOf { using type = GemvTail; };
template <> struct GemvTailOf<1> { using type = GemvTailEpi; };
template <> struct GemvTailOf<2> { using type = GemvTailEpi; };
// geom = nb | map << 16 | grid << 18  (nb < 2^16, grid < 2^14; checked by the launcher)

// Weight loads are plain global loads with clamped lane addresses; only the first XW waves load and
// quantize x (x-waves), the other waves issue their weight loads at once.  Two schedules (VAR):
// VAR 3:  the x-waves quantize, then issue their own weights (the x loads enter the CU's queue first)
// VAR 15: XFIRST + XHOLD: a workgroup barrier between the x-waves' x load ISSUE and every wave's
//         first weight issue, so the x loads are ahead of all of the workgroup's weight loads in the
//         CU's memory pipeline, and the x-waves issue their own weight loads only after x is in LDS
//         (round-2 phase stamps: without it the x data returned together with the weights, and the
//         prologue barrier gated compute).  The descriptor-load form and the all-waves prologue
//         (round 1) measured slower and are no longer built.
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

#ifdef GEMV_STAMPS
// diagnostic builds only (tools/build_variant.sh ... -DGEMV_STAMPS): per-wave s_memrealtime stamps of the
// launches whose M equals g_gemv_stamp_m: [wave][4] = start, x in LDS, end, HW_ID | XCC_ID << 32
__device__ uint64_t *g_gemv_stamps = nullptr;
__device__ int g_gemv_stamp_m = -1;
#endif
template <int NT, int WAVES, int DEPTH, int VAR, int PPL = 0, int PRO = 0, int BAL = 0, int EPI = 0>
__global__ __launch_bounds__(WAVES * 64) void k_gemv_q4_0(const float *__restrict__ x_, const uint8_t *W0,
                                                          const uint8_t *W1, const uint8_t *W2, int rb1_, int rb2_,
                                                          int rb3_, int rowbytes_, int geom, int M_,
                                                          const typename GemvTailOf<EPI>::type tail) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
#ifdef GEMV_STAMPS
    const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
#endif
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
        if constexpr (EPI == 2) {                                   // whole (gate, up) pairs per workgroup
            const uint32_t P = (uint32_t)M >> 1;
            row0 = 2 * (int)(((uint32_t)blockIdx.x * P) / (uint32_t)grid) + wave;
            rend = 2 * (int)(((uint32_t)(blockIdx.x + 1) * P) / (uint32_t)grid);
        } else {
            row0 = (int)(((uint32_t)blockIdx.x * (uint32_t)M) / (uint32_t)grid) + wave;
            rend = (int)(((uint32_t)(blockIdx.x + 1) * (uint32_t)M) / (uint32_t)grid);
        }
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

    static_assert(GEMV_MAXMAT == 4, "matrix selection below is written for 4 siblings");
    auto row_ptr = [&](int r) __attribute__((always_inline)) {     // wave-uniform
        if constexpr (EPI == 2)     // (gate, up) interleaved: row r is row r / 2 of matrix r & 1
            return reinterpret_cast<const uint8_t *>((uint64_t)w0 + ((r & 1) ? wd1 : 0)) + (int64_t)(r >> 1) * rowbytes;
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
#ifndef GEMV_XKO
#define GEMV_XKO 0          // diagnostic builds only (tools/build_variant.sh -DGEMV_XKO=n): x-prologue knockouts
#endif
    auto quantize_into_lds = [&](const u32x4 &raw, int t) __attribute__((always_inline)) {
#if GEMV_XKO >= 1           // 1: no quantize VALU (raw bits to LDS), 2: + a quarter of the x loads, 3: no x at all
        if (t < total) {
            xq[t] = raw.x ^ raw.w;
            if ((t & 7) == 0) {
                xd[t >> 3] = 1.0f;
                xs[t >> 3] = 0;
            }
        }
        return;
#endif
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
    constexpr bool XFIRST = (VAR & 4) != 0, XHOLD = (VAR & 8) != 0;
    static_assert(VAR == 3 || VAR == 15, "the production schedules");
    auto issue = [&](int it) __attribute__((always_inline)) {
        const bool valid = it < nitems;                             // past the end: one shared address
        const int r = valid ? item_row(it) : row0;
        ItemRegs v;
        const uint8_t *rp = row_ptr(valid ? r : 0);
#pragma unroll
        for (int j = 0; j < NPR; j++) {
            const int pp = 64 * (PPL > 0 ? j : item_chunk(it)) + lane;
            const int pc = valid ? (pp < npairs ? pp : npairs - 1) : 0;
            v.pr[j] = load_pair_g(rp + 36 * pc);
        }
        return v;
    };
    ItemRegs buf[DEPTH];
    if constexpr (PRO == 2) {
        // silu -> mul fused into the x prologue (NT == 1, one round of x-waves; see GemvNorm)
        static_assert(NT == 1, "silu prologue: decode x-wave form only");
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
            const bool store = blockIdx.x == 0;
#pragma unroll
            for (int i = 0; i < GEMV_XPRO; i++) {
                const int idx = tid + i * XT;
                if (idx < total) {
                    const uint32_t av[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
                    const uint32_t bv[4] = {rb[i].x, rb[i].y, rb[i].z, rb[i].w};
                    float u[4], o[4];
                    uint16_t hi[4], tv[4];           // indices first, then the lookups back to back
#pragma unroll
                    for (int c = 0; c < 4; c++) hi[c] = f2h(__uint_as_float(av[c]));
#pragma unroll
                    for (int c = 0; c < 4; c++) tv[c] = lut_silu(nrm.table, hi[c]);
#pragma unroll
                    for (int c = 0; c < 4; c++) {    // as k_silu_mul: s = table[fp16(a)], out = s * b
                        u[c] = h2f(tv[c]);
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
    } else if constexpr (PRO == 1) {
        // [add ->] rms_norm -> mul fused into the x prologue (NT == 1, one round of x-waves: the
        // launcher checks K <= 16 * 64 * 4 * GEMV_XPRO_N).  The x-waves hold the row in registers, sum
        // its squares in double (order-free in practice, as k_row_norm4's), exchange the per-wave
        // sums through LDS (one extra workgroup barrier), then scale, multiply by the norm weight and
        // quantize; workgroup 0 also stores the chain's tensors.
        static_assert(NT == 1, "norm prologue: decode x-wave form only");
        double *npart = reinterpret_cast<double *>(xs + NT * nb);
        const int XW = (total + 64 * GEMV_XPRO_N - 1) / (64 * GEMV_XPRO_N);
        const int XT = XW * 64;
        const GemvNorm nrm = tail.nrm;
        float4 v[GEMV_XPRO_N];
        u32x4 rg[GEMV_XPRO_N];                                   // the norm weight, loaded with x
        if (wave < XW) {
            const __amdgpu_buffer_rsrc_t ar = make_rsrc(nrm.a ? (const void *)nrm.a : (const void *)x,
                                                        nrm.a ? (uint32_t)total * 16u : 0u);
            const __amdgpu_buffer_rsrc_t gr = make_rsrc(nrm.w, (uint32_t)total * 16u);
            u32x4 rb[GEMV_XPRO_N], ra[GEMV_XPRO_N];
#pragma unroll
            for (int i = 0; i < GEMV_XPRO_N; i++) {
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
            for (int i = 0; i < GEMV_XPRO_N; i++) {
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
    } else {
        // x-waves: wave < XW load + quantize x (XT threads, PRO float4 each per round), then issue
        // their weight loads; the other waves only issue weight loads
        const int xtot = GEMV_XKO == 2 ? total / 4 : GEMV_XKO == 3 ? 0 : total;
        const int XW0 = (xtot + 64 * GEMV_XPRO - 1) / (64 * GEMV_XPRO);
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
            if (wave < XW) {
#pragma unroll
                for (int i = 0; i < GEMV_XPRO; i++) quantize_into_lds(xw[i], tid + i * XT);
                for (int base = GEMV_XPRO * XT; base < xtot; base += GEMV_XPRO * XT) {
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
            for (int base = 0; base < xtot; base += GEMV_XPRO * XT) {
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
#pragma unroll
            for (int d = 0; d < DEPTH; d++) buf[d] = issue(d);
        }
    }
    __syncthreads();
#ifdef GEMV_STAMPS
    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
#endif

    // ---- COMPUTE: stream the wave's items with DEPTH items in flight in a ring of named register
    // sets (no register copies: a copy would force a wait on the in-flight loads).
    float acc[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) acc[n] = 0.0f;
    float *const part = reinterpret_cast<float *>(xs + NT * nb);   // BAL: [rows of the WG][nchunk]
    // EPI: [row item][wave] outputs of the workgroup (after PRO 1's per-wave double sums)
    float *const epl = reinterpret_cast<float *>(xs + NT * nb) + (PRO == 1 ? 2 * WAVES : 0);
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
                const float2 dx = *reinterpret_cast<const float2 *>(xd + bA);
                const int2 sx = *reinterpret_cast<const int2 *>(xs + bA);
                const u32x4 *xc = reinterpret_cast<const u32x4 *>(xq + n * nb * 8) + p;
                const int sA = dot_q4_q8(qA0, qA1, qA2, qA3, xc[0], xc[npairs]) - sx.x;
                const int sB = dot_q4_q8(v.b.y, v.b.z, v.b.w, v.c, xc[2 * npairs], xc[3 * npairs]) - sx.y;
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
            if constexpr (EPI) {                                    // parked for the epilogue (NT == 1)
                if (lane == 0) epl[(it / nchunk) * WAVES + wave] = out;
            } else {
                if (lane < NT) yo[(int64_t)lane * ld] = out;
            }
        }
    };
    for (int it = 0; it < nitems; it += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            if (it + d >= nitems) break;
            process(buf[d], it + d);
            buf[d] = issue(it + d + DEPTH);
        }
    }
    if constexpr (EPI == 2) {
        // silu(gate) * up of the interleaved pairs, as k_silu_mul (its fp16 table value, then the product):
        // the even row's lane stores the gate output and silu(gate), the odd row's the up output and the product
        __syncthreads();
        if (lane < nrows_w) {
            typedef __attribute__((address_space(1))) float gfloat;
            const int k = lane;
            const int r = row0 + k * rstride;
            const float v = epl[k * WAVES + wave], pv = epl[k * WAVES + (wave ^ 1)];
            const bool odd = (r & 1) != 0;
            const float gate = odd ? pv : v, up = odd ? v : pv;
            const float u = h2f(lut_silu(tail.epi.table, f2h(gate)));
            const int e = r >> 1;
            float *const ym = reinterpret_cast<float *>(odd ? y0 + yd1 : y0);
            ((gfloat *)ym)[e] = v;
            float *const dst = odd ? tail.epi.d[1] : tail.epi.d[0];
            ((gfloat *)dst)[e] = odd ? u * up : u;
        }
    } else if constexpr (EPI) {
        // every output of the workgroup is in LDS: lane k of each wave finishes the wave's row k, pairing
        // row r with r ^ 1 (the same item of wave ^ 1 under the strided mapping, which the launcher enforces)
        static_assert(NT == 1 && PPL > 0 && !BAL, "epilogue: decode row items only");
        __syncthreads();
        if (lane < nrows_w) {
            typedef __attribute__((address_space(1))) float gfloat;
            typedef __attribute__((address_space(1))) uint16_t gu16;
            const int k = lane;
            const int r = row0 + k * rstride;
            const float v = epl[k * WAVES + wave], pv = epl[k * WAVES + (wave ^ 1)];
            const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
            const int mi = (int)g1 + (int)g2 + (int)g3;
            const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
            const uint32_t e = (uint32_t)(r - rb);
            float *const ym = reinterpret_cast<float *>(y0 + (g1 ? yd1 : 0) + (g2 ? yd2 : 0) + (g3 ? yd3 : 0));
            // this matrix's epilogue (constant-index field reads, selected per lane)
            const GemvEpi &ep = tail.epi;
            int kind = ep.kind[0], f16 = ep.f16[0], ne0 = ep.ne0[0], ne10 = ep.ne10[0], ne11 = ep.ne11[0];
            int nb10 = ep.nb10[0], nb11 = ep.nb11[0], nb12 = ep.nb12[0];
            float *d = ep.d[0];
            const float2 *cs = ep.cs[0];
            char *cc = ep.c[0];
#define GEMV_EPI_SEL(I)                                                                                      \
            if (mi == I) {                                                                                   \
                kind = ep.kind[I], f16 = ep.f16[I], ne0 = ep.ne0[I], ne10 = ep.ne10[I], ne11 = ep.ne11[I];   \
                nb10 = ep.nb10[I], nb11 = ep.nb11[I], nb12 = ep.nb12[I], d = ep.d[I], cs = ep.cs[I];          \
                cc = ep.c[I];                                                                                \
            }
            GEMV_EPI_SEL(1)
            GEMV_EPI_SEL(2)
            GEMV_EPI_SEL(3)
#undef GEMV_EPI_SEL
            float o = v;
            if (kind == 1) {                                        // rope mode 0, as k_elem_batch kind 0
                const uint32_t i0 = e - udiv20(e, (uint32_t)ne0) * (uint32_t)ne0;
                const float2 t = cs[i0 >> 1];
                o = (i0 & 1) ? pv * t.y + v * t.x : v * t.x - pv * t.y;
                ((gfloat *)d)[e] = o;
            }
            if (kind != 1 || d != ym) ((gfloat *)ym)[e] = v;        // the mul_mat's own output
            if (cc) {                                               // linear element e of the copy's view
                const uint32_t q10 = udiv20(e, (uint32_t)ne10), i10 = e - q10 * (uint32_t)ne10;
                const uint32_t i12 = udiv20(q10, (uint32_t)ne11), i11 = q10 - i12 * (uint32_t)ne11;
                char *dst = cc + (int64_t)i10 * nb10 + (int64_t)i11 * nb11 + (int64_t)i12 * nb12;
                if (f16)
                    *(gu16 *)dst = (uint16_t)f2h(o);
                else
                    *(gfloat *)dst = o;
            }
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
#ifdef GEMV_STAMPS
    if (M == g_gemv_stamp_m && g_gemv_stamps && lane == 0) {      // vector stores (lane-divergent)
        const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);          // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);        // HW_REG_XCC_ID
        volatile uint64_t *st = g_gemv_stamps + ((int64_t)blockIdx.x * WAVES + wave) * 4;
        st[0] = ts0;
        st[1] = ts1;
        st[2] = ts2;
        st[3] = (uint64_t)hw | ((uint64_t)xcc << 32);
    }
#endif
}


#ifdef GEMV_STAMPS
extern "C" int ggml_hip_debug_gemv_stamps(void *buf, int m) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_gemv_stamps), &buf, sizeof(buf)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_gemv_stamp_m), &m, sizeof(m)) != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif

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


template <int NT, int WAVES, int DEPTH, int VAR, int PPL = 0, int PRO = 0, int BAL = 0, int EPI = 0>
static hipError_t launch_gemv_w(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s,
                                const GemvNorm *nrm = nullptr, const GemvEpi *epi = nullptr) {
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
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_occ, k_gemv_q4_0<NT, WAVES, DEPTH, VAR, PPL, PRO, BAL, EPI>,
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
    if (EPI) {
        // strided rows (row r ^ 1 is the same item of wave ^ 1 in the same workgroup) or, for the
        // interleaved (gate, up) rows, blocked whole pairs per workgroup; every output of the workgroup
        // parked in LDS, pairs never straddling two matrices
        map = EPI == 2 && map_env != 0 ? 2 : 0;     // GGML_HIP_GEMV_MAP=0: strided pairs for w1|w3 too
        if (EPI == 2 && (m.n != 2 || 2 * m.row_begin[1] != m.row_begin[2])) return hipErrorInvalidValue;
        for (int i = 1; i <= m.n; i++)
            if (m.row_begin[i] & 1) return hipErrorInvalidValue;
        if (map == 2 && (int64_t)grid * M >= (int64_t)1 << 32) return hipErrorInvalidValue;
        const int64_t rows_w = map == 2 ? (2 * ((M / 2 + grid - 1) / grid) + WAVES - 1) / WAVES
                                        : (M + (int64_t)grid * WAVES - 1) / ((int64_t)grid * WAVES);
        lds += (size_t)rows_w * WAVES * sizeof(float);
        if (lds > GEMV_LDS_MAX || rows_w > 64) return hipErrorInvalidValue;   // one lane per row of a wave
    }
    if (nb >= (1 << 16) || grid >= (1u << 14) || rowbytes > INT_MAX || M > INT_MAX) return hipErrorInvalidValue;
    typename GemvTailOf<EPI>::type tail{};
    if constexpr (EPI) tail.epi = *epi;
    if (nrm) tail.nrm = *nrm;
    tail.W3 = m.W[3];
    for (int i = 0; i < GEMV_MAXMAT; i++) {
        tail.y[i] = m.y[i];
        tail.ldy[i] = m.ldy[i];
    }
    const int geom = nb | map << 16 | (int)(grid << 18);
    (void)hipGetLastError();  // report only this launch's error
    launch_k((k_gemv_q4_0<NT, WAVES, DEPTH, VAR, PPL, PRO, BAL, EPI>), dim3(grid), dim3(WAVES * 64), lds, s, x, m.W[0],
                       m.W[1], m.W[2], m.row_begin[1], m.row_begin[2], m.row_begin[3], (int)rowbytes, geom, (int)M, tail);
    return hipGetLastError();
}

template <int NT, int VAR>
static hipError_t launch_gemv_rows(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s,
                                   int ppl, int rd) {
    switch (ppl) {
        case 1: return rd == 1 ? launch_gemv_w<NT, GEMV_WAVES, 1, VAR, 1>(m, K, x, dev, s)
                               : launch_gemv_w<NT, GEMV_WAVES, 2, VAR, 1>(m, K, x, dev, s);
        case 2: return rd == 1 ? launch_gemv_w<NT, GEMV_WAVES, 1, VAR, 2>(m, K, x, dev, s)
                               : launch_gemv_w<NT, GEMV_WAVES, 2, VAR, 2>(m, K, x, dev, s);
        default: return rd == 1 ? launch_gemv_w<NT, GEMV_WAVES, 1, VAR, 3>(m, K, x, dev, s)
                                : launch_gemv_w<NT, GEMV_WAVES, 2, VAR, 3>(m, K, x, dev, s);
    }
}

template <int NT>
static hipError_t launch_gemv(const GemvMats &m, int64_t K, const float *x, const DeviceInfo &dev, hipStream_t s) {
    // VAR 3 or 15 (policy below), decode row items at ring depth 1; chunked items (N > 1 or K > 12288)
    // at depth 1 for single-chunk rows and 2 otherwise (measured per shape, tools/gemv_ab.sh).
    // GGML_HIP_GEMV_VAR=3|15 and GGML_HIP_GEMV_DEPTH=1|2 force the alternatives (same y bitwise).
    static const int var_env = env_int("GGML_HIP_GEMV_VAR", -1);
    const int depth_env = gemv_policy().depth;
    // Decode row items (round 2, with preloaded kernargs; tools/gemv_ab.sh, LLaMA-7B shapes): one row
    // in flight per wave, and XHOLD (VAR 15: the x-waves issue their own weights once x is in LDS)
    // when a wave has at most two rows and x is short (wq|wk|wv 7.33 -> 7.19 us, wo 4.82 -> 4.24);
    // VAR 3 otherwise (w1|w3 at 2.7 rows per wave 10.56 vs 10.73, w2 at K = 11008 7.33 vs 8.06)
    const int64_t Mrows = m.row_begin[m.n];
    const int var = var_env == 3 || var_env == 15
                        ? var_env : (NT == 1 && K <= 8192 && Mrows <= 2 * 16 * (int64_t)dev.num_cus * 2 ? 15 : 3);
    const int depth = depth_env ? depth_env : (K / 64 > 64 ? 2 : 1);
    if constexpr (NT == 1) {                        // decode: one item per row (PPL pairs per lane)
        const int rowitems = gemv_policy().rowitems;
        const int ppl = (int)((K / 64 + 63) / 64);
        if (rowitems && ppl <= 3) {
            const int rd = depth_env ? depth_env : 1;
            return var == 15 ? launch_gemv_rows<NT, 15>(m, K, x, dev, s, ppl, rd)
                             : launch_gemv_rows<NT, 3>(m, K, x, dev, s, ppl, rd);
        }
        // K > 12288: chunked items below (measured equal or faster at 4-5 pairs per lane), balanced at
        // chunk granularity (BAL) when whole rows per wave leave a long tail: the busiest wave of the
        // row-granular mapping streams ceil(M / waves) rows, a BAL wave ceil(rows per WG * chunks / 16)
        // chunks; BAL when that is at most 0.65 of the rows' chunks (GGML_HIP_GEMV_BAL=0/1 overrides).
        // Measured (tools/r2_bal.sh, 2 rounds): Falcon 18176 -> 4544 14.6 -> 13.2-14.1 us (the bench's
        // Falcon-7B line 845 -> 875 tok/s), LLaMA-13B 13824 -> 5120 11.25 either way, NeoX 24576 -> 6144
        // 20.2 -> 20.9-21.1 (0.75: not taken)
        const int bal_env = gemv_policy().bal;
        if (var == 3 && bal_env != 0 && ppl > 3) {
            const int64_t cus = dev.num_cus;
            const int64_t wg = gemv_policy().wg_per_cu > 0 ? gemv_policy().wg_per_cu : (Mrows <= 2 * cus * 16 ? 1 : 2);
            const int64_t need = (Mrows + 15) / 16, cap = cus * wg;        // launch_gemv_w's grid rule
            const int64_t bgrid = need <= cus ? need : cus * ((need + cus - 1) / cus);
            const int64_t grid = bgrid < cap ? bgrid : cap, nchunk = (K / 64 + 63) / 64;
            const int64_t rows_w = (Mrows + grid * 16 - 1) / (grid * 16);
            const int64_t items_w = (((Mrows + grid - 1) / grid) * nchunk + 15) / 16;
            const int64_t lds_bal = (K / QK) * 40 + ((Mrows + grid - 1) / grid) * nchunk * 4;
            if (lds_bal <= GEMV_LDS_MAX && (bal_env == 1 || 20 * items_w <= 13 * rows_w * nchunk))
                return depth == 1 ? launch_gemv_w<NT, GEMV_WAVES, 1, 3, 0, 0, 1>(m, K, x, dev, s)
                                  : launch_gemv_w<NT, GEMV_WAVES, 2, 3, 0, 0, 1>(m, K, x, dev, s);
        }
    }
    return depth == 1 ? launch_gemv_w<NT, GEMV_WAVES, 1, 3>(m, K, x, dev, s)
                      : launch_gemv_w<NT, GEMV_WAVES, 2, 3>(m, K, x, dev, s);
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
                                   const GemvNorm &nrm, int rd, const GemvEpi *epi) {
    if (epi) {                           // the q|k|v or w1|w3 epilogue: rms_norm prologue, ring depth 1 (same y)
        if (nrm.kind != 1) return hipErrorInvalidValue;
        return epi->glu ? launch_gemv_w<1, GEMV_WAVES, 1, VAR, PPL, 1, 0, 2>(m, K, b, dev, s, &nrm, epi)
                        : launch_gemv_w<1, GEMV_WAVES, 1, VAR, PPL, 1, 0, 1>(m, K, b, dev, s, &nrm, epi);
    }
    if (nrm.kind == 2)
        return rd == 2 ? launch_gemv_w<1, GEMV_WAVES, 2, VAR, PPL, 2>(m, K, b, dev, s, &nrm)
                       : launch_gemv_w<1, GEMV_WAVES, 1, VAR, PPL, 2>(m, K, b, dev, s, &nrm);
    return rd == 2 ? launch_gemv_w<1, GEMV_WAVES, 2, VAR, PPL, 1>(m, K, b, dev, s, &nrm)
                   : launch_gemv_w<1, GEMV_WAVES, 1, VAR, PPL, 1>(m, K, b, dev, s, &nrm);
}

hipError_t gemv_q4_0_multi_norm(int nmat, const void *const *W, const int64_t *M, int64_t K, const float *b,
                                const GemvNorm &nrm, float *const *y, const int64_t *ldy, const DeviceInfo &dev,
                                hipStream_t s, const GemvEpi *epi) {
    // one round of x-waves holds the row: K / 4 float4 <= 16 waves * 64 lanes * GEMV_XPRO
    if (nmat < 1 || nmat > GEMV_MAXMAT || K % 64 != 0 || K / 4 > 16 * 64 * (nrm.kind == 1 ? GEMV_XPRO_N : GEMV_XPRO) || !b ||
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
        if (ppl == 1) return launch_gemv_norm<15, 1>(m, K, b, dev, s, nrm, rd, epi);
        if (ppl == 2) return launch_gemv_norm<15, 2>(m, K, b, dev, s, nrm, rd, epi);
        if (ppl == 3) return launch_gemv_norm<15, 3>(m, K, b, dev, s, nrm, rd, epi);
    } else {
        if (ppl == 1) return launch_gemv_norm<3, 1>(m, K, b, dev, s, nrm, rd, epi);
        if (ppl == 2) return launch_gemv_norm<3, 2>(m, K, b, dev, s, nrm, rd, epi);
        if (ppl == 3) return launch_gemv_norm<3, 3>(m, K, b, dev, s, nrm, rd, epi);
    }
    return hipErrorInvalidValue;        // K > 12288: chunked items are not instantiated with the prologue
}

}  // namespace ghip
