// q4_0_engine.hip — the persistent decode engine: a chain of dependent N = 1 q4_0 mul_mats (the decode's
// wq|wk|wv -> wo -> w1|w3 -> w2 -> next layer ..., llama.cpp:1334-1500 -> ggml_compute_forward_mul_mat_q_f32,
// ggml.c:11353-11411, once per mul_mat) as ONE launch of one workgroup per CU.
//
// Why: the per-launch decode GEMV streams at ~6.5 TB/s but pays ~2.8 us of fixed cost per
// launch (boundary, dispatch ramp, first-byte latency, tail) — 4 launches per LLaMA layer, 0.48 of HBM
// peak.  Two earlier in-launch designs lost because the hand-off's own memory operations (flag polls, x
// loads, y stores) queued behind the next matrix's bulk weight loads in the CU's memory pipeline.  This
// engine is the MI355X guide's weight-streaming engine (MI355X_MICROARCH.md, price rows ldsdma-fill,
// prefetch-credit, allgather, engine-vs-launches): per CU
//   * ONE loader wave streams the CU's weight rows, in the order the CU will consume them, into a 128 KiB
//     LDS ring by LDS-DMA (global_load_lds_dwordx4: no VGPR destination, nothing for the compiler to wait
//     on), ENG_D lines of 1 KiB in flight, running ahead ACROSS dependency edges: while the chip waits for
//     the last producer of an op, every ring already holds the next op's first rows;
//   * ENG_NC consumer waves compute the rows out of the ring with the decode GEMV's exact per-row
//     arithmetic (lane p: block pair p, p+64, p+128; v_dot4c on unsigned nibbles, -8*sum(q) per block, fp32
//     fma chain over the lane's pairs, the same DPP tree) — so every y is bitwise the per-launch GEMV's;
//   * the all-to-all edge is carried by q8_0 granules: the CU that completes a 32-row unit of an output that
//     the next task reads quantizes it ONCE (q8_block_lane, the same bits as the GEMV's x prologue) and
//     publishes the block as 8 aligned 8-byte {tag16 | aux16 | 4 int8} granules with agent-scope stores
//     (aux = fp16 d in word 0, sum(q) in word 1); consumer wave 0 of each CU sweeps the granules of the x it
//     needs into LDS (tag = this launch's epoch, so stale granules of the previous launch never match), and
//     the consumer waves load x into registers once per task.
// Work split (host, engine_plan_create): every matrix in units of 32 rows (one q8_0 block of its output),
// units dealt in task order to the least-loaded CU (cumulative bytes), the units of the output the next
// task reads first within a task, so that edge fires while the rest of the task is still streaming.
//
// Every wait is bounded (s_memrealtime, 100 MHz; timeout argument): a wait that expires sets the CU's abort
// flag and an error bit in the control block, every wave of the CU drains, the launch ends, and
// ggml_hip_chain_status reports it.  The launch needs all of its workgroups co-resident (one per CU: the
// LDS footprint admits one), i.e. no concurrent kernel on the device.
#include "q4_0_device.h"

#include <algorithm>
#include <queue>
#include <string>
#include <vector>

#include "../../include/ggml-hip.h"

namespace ghip {

#ifndef ENG_NC_DEF
#define ENG_NC_DEF 8
#endif
#ifndef ENG_PRIO
#define ENG_PRIO 0          // the loader wave's s_setprio (variants)
#endif
#ifndef ENG_G_DEF
#define ENG_G_DEF 16
#endif
#ifndef ENG_THIN
#define ENG_THIN 0          // lines the loader keeps in flight while its CU sweeps granules (0: not thinned)
#endif
#ifndef ENG_SLEEP
#define ENG_SLEEP 1         // s_sleep argument of the consumers' spin steps
#endif
// consumer waves (wave ENG_NC is the loader): a consumer row is a serial chain of LDS reads, VALU, a DPP tree and
// the output store (~500+ cycles), so rows in flight need waves: 4 consumers (one per SIMD) retired ~18 GB/s per
// CU, below the loader's stream
constexpr int ENG_NC = ENG_NC_DEF;
constexpr int ENG_THREADS = (ENG_NC + 1) * 64;
constexpr uint32_t ENG_RING = 128u * 1024u;     // LDS ring (power of two)
constexpr uint32_t ENG_LINE = 1024u;            // one LDS-DMA instruction: 64 lanes x 16 B
constexpr int ENG_D = 40;                       // lines in flight per loader (vmcnt <= 63)
constexpr int ENG_G = ENG_G_DEF;                // lines per loader step (control work once per step)
constexpr int ENG_MAXNB = 384;                  // K <= 12288 (3 block pairs per lane)
constexpr int ENG_SLOTS = 16;                   // park slots of consumed units (32 floats each)
// LDS layout (bytes)
constexpr uint32_t L_XQ = ENG_RING;                           // x q8 ints, chunk-major [4][npairs][16 B]
constexpr uint32_t L_XD = L_XQ + ENG_MAXNB * 32;              // float [nb]: h2f(d16)
constexpr uint32_t L_XS = L_XD + ENG_MAXNB * 4;               // int [nb]: 8 * sum(q)
constexpr uint32_t L_PAR = L_XS + ENG_MAXNB * 4;              // float [SLOTS][32]
constexpr uint32_t L_CTL = L_PAR + ENG_SLOTS * 32 * 4;        // uint32 control words
enum { C_LANDED = 0, C_XGEN = 1, C_XLOADED = 2, C_ABORT = 3, C_PROG = 4, C_CNT = 20, C_QDONE = 36, C_GATHER = 52,
       C_WORDS = 56 };
constexpr uint32_t ENG_LDS = L_CTL + C_WORDS * 4;
static_assert(ENG_LDS <= 160 * 1024, "engine LDS");
static_assert(ENG_NC >= 1 && ENG_NC <= 12 && C_PROG + 16 <= C_CNT && C_CNT + ENG_SLOTS <= C_QDONE &&
              C_QDONE + ENG_SLOTS <= C_WORDS, "ctl words");

// error bits (ctl[2]); ctl[3] = the first timeout's site (CU << 8 | code)
enum { ENG_E_LOADER = 1, ENG_E_LANDED = 2, ENG_E_XGEN = 4, ENG_E_GATHER = 8, ENG_E_SLOT = 16, ENG_E_XLOADED = 32 };

struct EngTask {
    const float *xext;          // x read from memory (task 0), or nullptr
    const uint64_t *xgran;      // x from the granules of the previous task's consumed output, or nullptr
    float *y[4];
    uint64_t *gran[4];          // granules of output i when the next task reads it, else nullptr
    uint32_t K, nb, npairs, rowbytes;
};
struct EngUnit {                // 32 B, read with scalar loads
    uint32_t src_lo, src_hi;    // address of the unit's first row
    uint32_t soff;              // offset in the CU's stream (multiple of ENG_LINE)
    uint32_t bytes;             // nrows * rowbytes
    uint32_t row0;              // first row within its matrix
    uint32_t rbase;             // CU-local index of the unit's first row (rows go round-robin to the consumers)
    uint32_t cidx;              // ordinal among the CU's consumed units (park slot cidx % SLOTS), ~0u: not consumed
    uint32_t tmn;               // task | mat << 16 | nrows << 24
};
struct EngCU {
    uint32_t unit0, nunits, stream_bytes, pad;
};
struct EngArgs {
    const EngTask *tasks;
    const EngUnit *units;
    const EngCU *cus;
    uint64_t *ctl;              // [0] epoch, [1] arrivals, [2] error bits, [3] first error site
    uint32_t timeout;           // ticks of s_memrealtime
    uint32_t diag;              // diagnostics only (GGML_HIP_ENGINE_DIAG): 1 the gather takes granules unchecked,
                                // 2 the consumers skip the row arithmetic, 4 no y stores of unconsumed rows
                                // (results wrong in all three)
    uint64_t *stamps;           // diagnostics only (GGML_HIP_ENGINE_STAMPS=1): per CU ENG_ST_HDR header words +
                                // ENG_ST_TASKS x ENG_ST_W per-task stamps, or nullptr: [0] wave 0 starts the task
                                // (gather), [1] x in LDS, [2] wave 0's last row, [3] task id, [4] the CU's last
                                // granule publish of the task (max), [5] wave 0's first row consumed
};
constexpr int ENG_ST_HDR = 8, ENG_ST_TASKS = 160, ENG_ST_W = 6, ENG_ST_CU = ENG_ST_HDR + ENG_ST_W * ENG_ST_TASKS;

typedef __attribute__((address_space(1))) uint64_t g_u64;
// the tables are read through the constant address space: wave-uniform scalar loads (SMEM) that neither wait
// behind the loader's vector-memory queue nor count in vmcnt
typedef __attribute__((address_space(4))) const EngUnit c_unit;
typedef __attribute__((address_space(4))) const EngTask c_task;
typedef __attribute__((address_space(4))) const EngCU c_cu;
__device__ __forceinline__ EngUnit ld_unit(const EngUnit *base, uint32_t i) {
    const c_unit *u = (const c_unit *)base + i;
    EngUnit r;
    r.src_lo = u->src_lo;
    r.src_hi = u->src_hi;
    r.soff = u->soff;
    r.bytes = u->bytes;
    r.row0 = u->row0;
    r.rbase = u->rbase;
    r.cidx = u->cidx;
    r.tmn = u->tmn;
    return r;
}
__device__ __forceinline__ EngTask ld_task(const EngTask *base, uint32_t i) {
    const c_task *t = (const c_task *)base + i;
    EngTask r;
    r.xext = t->xext;
    r.xgran = t->xgran;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        r.y[k] = t->y[k];
        r.gran[k] = t->gran[k];
    }
    r.K = t->K;
    r.nb = t->nb;
    r.npairs = t->npairs;
    r.rowbytes = t->rowbytes;
    return r;
}
__device__ __forceinline__ EngCU ld_cu(const EngCU *base, uint32_t i) {
    const c_cu *c = (const c_cu *)base + i;
    EngCU r;
    r.unit0 = c->unit0;
    r.nunits = c->nunits;
    r.stream_bytes = c->stream_bytes;
    r.pad = 0;
    return r;
}

// ---- LDS access of the loader wave: inline asm only, so that the compiler's waitcnt pass (which sees
// nothing of the asm LDS-DMA) never inserts a vmcnt wait before them
__device__ __forceinline__ void eng_dma(const void *gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}
__device__ __forceinline__ u32x4 eng_ld4_asm(uint32_t addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
// the consumers' minimum progress (loader): the NC words by ds_read_b128
__device__ __forceinline__ uint32_t eng_min_prog(uint32_t addr) {
    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < (ENG_NC + 3) / 4; q++) {     // the words past NC hold ~0 (kernel start)
        const u32x4 pg = eng_ld4_asm(addr + 16 * q);
        m = min(m, min(min(pg.x, pg.y), min(pg.z, pg.w)));
    }
    return __builtin_amdgcn_readfirstlane(m);
}

__device__ __forceinline__ uint32_t eng_ld_asm(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
__device__ __forceinline__ void eng_st_asm(uint32_t addr, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
// consumer-side control words: relaxed workgroup-scope LDS atomics (no vmcnt waits)
__device__ __forceinline__ uint32_t cld(uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void cst(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

__device__ __forceinline__ void eng_fail(const EngArgs &a, uint32_t *ctl, uint32_t code) {
    cst(ctl + C_ABORT, 1u);
    __hip_atomic_fetch_or(a.ctl + 2, (uint64_t)code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t z = 0;
    __hip_atomic_compare_exchange_strong(a.ctl + 3, &z, (uint64_t)blockIdx.x << 8 | code, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one bounded spin step: false when this CU aborts (its own timeout or another wave's)
__device__ __forceinline__ bool eng_spin(const EngArgs &a, uint32_t *ctl, uint64_t t0, uint32_t code) {
    if (cld(ctl + C_ABORT)) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
        eng_fail(a, ctl, code);
        return false;
    }
    __builtin_amdgcn_s_sleep(ENG_SLEEP);
    return true;
}

// p[i] for a wave-uniform i < 4 as selects (a runtime index into a by-value array puts the array in scratch)
template <typename P> __device__ __forceinline__ P sel4(const P (&p)[4], uint32_t i) {
    return i == 0 ? p[0] : i == 1 ? p[1] : i == 2 ? p[2] : p[3];
}

template <int PPL> struct EngX {
    u32x4 c0[PPL], c1[PPL], c2[PPL], c3[PPL];   // block A words 0-3, 4-7; block B words 0-3, 4-7
    float2 d[PPL];
    int2 s[PPL];
};

// one weight row out of the ring: the GEMV's per-lane pair loop (q4_0_gemv.hip process()) and reduction
template <int PPL>
__device__ __forceinline__ float eng_row(const uint32_t *ring, uint32_t rb, bool wraps, const EngX<PPL> &x,
                                         int npairs, int lane) {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < PPL; j++) {
        const int p = lane + 64 * j;
        if (p < npairs) {
            const uint32_t a = rb + 36u * (uint32_t)p;
            uint32_t w[9];
            if (!wraps) {
                const uint32_t *q = ring + (a >> 2);
#pragma unroll
                for (int k = 0; k < 9; k++) w[k] = q[k];
            } else {
#pragma unroll
                for (int k = 0; k < 9; k++) w[k] = ring[((a + 4u * k) & (ENG_RING - 1)) >> 2];
            }
            const float dA = h2f(w[0] & 0xFFFFu);
            const float dB = h2f(w[4] >> 16);
            const uint32_t qA0 = __builtin_amdgcn_alignbyte(w[1], w[0], 2);
            const uint32_t qA1 = __builtin_amdgcn_alignbyte(w[2], w[1], 2);
            const uint32_t qA2 = __builtin_amdgcn_alignbyte(w[3], w[2], 2);
            const uint32_t qA3 = __builtin_amdgcn_alignbyte(w[4], w[3], 2);
            const uint32_t m = 0x0F0F0F0Fu;
            int sA = 0, sB = 0;
            sA = __builtin_amdgcn_sdot4((int)(qA0 & m), (int)x.c0[j].x, sA, false);
            sA = __builtin_amdgcn_sdot4((int)(qA1 & m), (int)x.c0[j].y, sA, false);
            sA = __builtin_amdgcn_sdot4((int)(qA2 & m), (int)x.c0[j].z, sA, false);
            sA = __builtin_amdgcn_sdot4((int)(qA3 & m), (int)x.c0[j].w, sA, false);
            sA = __builtin_amdgcn_sdot4((int)((qA0 >> 4) & m), (int)x.c1[j].x, sA, false);
            sA = __builtin_amdgcn_sdot4((int)((qA1 >> 4) & m), (int)x.c1[j].y, sA, false);
            sA = __builtin_amdgcn_sdot4((int)((qA2 >> 4) & m), (int)x.c1[j].z, sA, false);
            sA = __builtin_amdgcn_sdot4((int)((qA3 >> 4) & m), (int)x.c1[j].w, sA, false);
            sB = __builtin_amdgcn_sdot4((int)(w[5] & m), (int)x.c2[j].x, sB, false);
            sB = __builtin_amdgcn_sdot4((int)(w[6] & m), (int)x.c2[j].y, sB, false);
            sB = __builtin_amdgcn_sdot4((int)(w[7] & m), (int)x.c2[j].z, sB, false);
            sB = __builtin_amdgcn_sdot4((int)(w[8] & m), (int)x.c2[j].w, sB, false);
            sB = __builtin_amdgcn_sdot4((int)((w[5] >> 4) & m), (int)x.c3[j].x, sB, false);
            sB = __builtin_amdgcn_sdot4((int)((w[6] >> 4) & m), (int)x.c3[j].y, sB, false);
            sB = __builtin_amdgcn_sdot4((int)((w[7] >> 4) & m), (int)x.c3[j].z, sB, false);
            sB = __builtin_amdgcn_sdot4((int)((w[8] >> 4) & m), (int)x.c3[j].w, sB, false);
            sA -= x.s[j].x;
            sB -= x.s[j].y;
            acc = fmaf((float)sA, dA * x.d[j].x, acc);
            acc = fmaf((float)sB, dB * x.d[j].y, acc);
        }
    }
    const float t = wave_sum_lane63(acc);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 63));
}

// the consumers' part of one task: x registers from LDS, then the rows of the CU's units of the task
template <int PPL>
__device__ __forceinline__ void eng_task_rows(const EngArgs &a, uint32_t *ctl, const uint32_t *ring, float *par,
                                              const EngTask &tk, uint32_t &ui, uint32_t uend, uint32_t task, int w,
                                              int lane, uint32_t tag, bool &abort, uint64_t *sk) {
    bool first_row = true;
    const uint32_t *xq = ring + L_XQ / 4;
    const float *xd = reinterpret_cast<const float *>(ring + L_XD / 4);
    const int *xs = reinterpret_cast<const int *>(ring + L_XS / 4);
    const int npairs = (int)tk.npairs;
    EngX<PPL> x;
#pragma unroll
    for (int j = 0; j < PPL; j++) {
        const int p = lane + 64 * j;
        const int pc = p < npairs ? p : 0;
        const u32x4 *xc = reinterpret_cast<const u32x4 *>(xq) + pc;
        x.c0[j] = xc[0];
        x.c1[j] = xc[npairs];
        x.c2[j] = xc[2 * npairs];
        x.c3[j] = xc[3 * npairs];
        x.d[j] = *reinterpret_cast<const float2 *>(xd + 2 * pc);
        x.s[j] = *reinterpret_cast<const int2 *>(xs + 2 * pc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(ctl + C_XLOADED, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    typedef __attribute__((address_space(1))) float gfloat;
    // the next unit's descriptor is loaded while this one's rows run (a scalar-cache miss per unit otherwise
    // stalls the wave ahead of its first row); landed is re-read only when a row lies past the value last seen
    EngUnit Un = ld_unit(a.units, ui);
    uint32_t lnd = 0;
    for (; ui < uend; ui++) {
        const EngUnit U = Un;
        if (ui + 1 < uend) Un = ld_unit(a.units, ui + 1);
        const uint32_t tmn = U.tmn;
        if ((tmn & 0xFFFFu) != task) break;
        const uint32_t mat = (tmn >> 16) & 0xFFu, nrows = tmn >> 24;
        const bool consumed = U.cidx != ~0u;
        const uint32_t slot = consumed ? U.cidx % ENG_SLOTS : 0, gen = consumed ? U.cidx / ENG_SLOTS : 0;
        // this wave's first row of the unit: rows go round-robin by CU-local row index
        uint32_t r = (uint32_t)((w - (int)(U.rbase % ENG_NC) + ENG_NC) % ENG_NC);
        if (consumed && r < nrows) {             // the park slot's previous unit must have been quantized
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (cld(ctl + C_QDONE + slot) < gen)
                if (!eng_spin(a, ctl, t0, ENG_E_SLOT)) { abort = true; return; }
        }
        for (; r < nrows; r += ENG_NC) {
            const uint32_t start = U.soff + r * tk.rowbytes, end = start + tk.rowbytes;
            if (lnd < end) lnd = cld(ctl + C_LANDED);
            if (lnd < end) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while ((lnd = cld(ctl + C_LANDED)) < end)
                    if (!eng_spin(a, ctl, t0, ENG_E_LANDED)) { abort = true; return; }
                if (a.stamps && w == 0 && lane == 0)           // wave 0's ticks waiting for landed lines
                    a.stamps[(uint64_t)blockIdx.x * ENG_ST_CU + 3] += __builtin_amdgcn_s_memrealtime() - t0;
            }
            asm volatile("" ::: "memory");
            const uint32_t rb = start & (ENG_RING - 1);
            const float out = (a.diag & 2) ? 0.0f : eng_row<PPL>(ring, rb, rb + tk.rowbytes > ENG_RING, x, npairs, lane);
            if (sk && first_row && w == 0 && lane == 0) sk[5] = __builtin_amdgcn_s_memrealtime();
            first_row = false;
            if (consumed) {
                if (lane == 0) par[slot * 32 + r] = out;
                uint32_t old = 0;
                if (lane == 0) old = __hip_atomic_fetch_add(ctl + C_CNT + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                old = __builtin_amdgcn_readfirstlane(old);
                asm volatile("" ::: "memory");   // the parked rows are read only after the count said so
                if (old + 1 == nrows) {          // the unit's last row: quantize the block once, publish it
                    const int l8 = lane & 7;
                    const float4 v = reinterpret_cast<const float4 *>(par + slot * 32)[l8];
                    uint32_t d16;
                    int qsum;
                    const uint32_t packed = q8_block_lane(v, d16, qsum);
                    if (lane < 8) {
                        const uint32_t aux = lane == 0 ? d16 : lane == 1 ? ((uint32_t)qsum & 0xFFFFu) : 0u;
                        const uint64_t g = (uint64_t)tag << 48 | (uint64_t)aux << 32 | packed;
                        g_u64 *gp = (g_u64 *)(sel4(tk.gran, mat) + (U.row0 >> 5) * 8 + lane);
                        __hip_atomic_store(gp, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // one sc1 store
                        gfloat *yo = (gfloat *)(sel4(tk.y, mat) + U.row0 + 4 * lane);
                        yo[0] = v.x;
                        yo[1] = v.y;
                        yo[2] = v.z;
                        yo[3] = v.w;
                    }
                    if (sk && lane == 0)
                        __hip_atomic_fetch_max(sk + 4, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    if (lane == 0) {
                        cst(ctl + C_CNT + slot, 0u);
                        __hip_atomic_fetch_add(ctl + C_QDONE + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            } else if (lane == 0 && !(a.diag & 4)) {
                ((gfloat *)sel4(tk.y, mat))[U.row0 + r] = out;
            }
            if (lane == 0) cst(ctl + C_PROG + w, end);
        }
    }
}

__global__ __launch_bounds__(ENG_THREADS) void k_engine_q4_0(const EngArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t elds[];
    uint32_t *ring = elds;
    uint32_t *ctl = elds + L_CTL / 4;
    float *par = reinterpret_cast<float *>(elds + L_PAR / 4);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const EngCU cu = ld_cu(a.cus, blockIdx.x);
    // tag of this launch: the epoch (advanced by the last workgroup of the previous launch), 1..65535
    const uint32_t epoch = (uint32_t)__hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tag = epoch % 65535u + 1u;
    if (tid < C_WORDS) ctl[tid] = (tid >= C_PROG + ENG_NC && tid < C_PROG + 16) ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t *)elds);   // ring's LDS address

    uint64_t *st = a.stamps ? a.stamps + (uint64_t)blockIdx.x * ENG_ST_CU : nullptr;
    if (w == ENG_NC) {
        // ---------------- loader: the CU's stream, line by line, into the ring
        if (ENG_PRIO) __builtin_amdgcn_s_setprio(ENG_PRIO);
        const uint64_t tl0 = __builtin_amdgcn_s_memrealtime();
        uint64_t ring_wait = 0;
        const uint32_t nlines = (cu.stream_bytes + ENG_LINE - 1) / ENG_LINE;
        uint32_t ui = cu.unit0;
        const uint32_t uend_i = cu.unit0 + cu.nunits;
        uint32_t uend_b = 0, usoff = 0;
        __amdgpu_buffer_rsrc_t urs = make_rsrc(nullptr, 0);
        EngUnit Un{};                              // the next unit's descriptor, loaded one unit ahead
        if (cu.nunits) Un = ld_unit(a.units, ui);
        uint32_t issued = 0, pub = 0;              // lines issued; landed bytes published (monotonic)
        uint32_t freed = 0;                        // the consumers' progress as last read (rows before it are done)
        bool ok = true;
        // The loop's per-line cost IS the stream rate (a 1 KiB line every ~50 ns per CU at 20 GB/s): every control
        // step (ring-space check, landed publication) runs once per group of ENG_G lines, the lines themselves
        // are a compare + the DMA (tools/ldsdma_mb.hip: one LDS read + lgkmcnt wait per line halved the rate)
        for (uint32_t g0 = 0; g0 < nlines && ok; g0 += ENG_G) {
            const uint32_t gn = min((uint32_t)ENG_G, nlines - g0);
            const uint32_t gend = (g0 + gn) * ENG_LINE;
            // ring space for the whole group: every consumer past gend - RING
            if (gend > ENG_RING && gend - ENG_RING > freed) {
                const uint32_t need = gend - ENG_RING;
                // (every value read by the asm is made wave-uniform: a VGPR result in a loop condition makes the
                // compiler treat the unit descriptors as divergent, load them with vector loads and drain the DMAs)
                freed = eng_min_prog(lds0 + L_CTL + C_PROG * 4);
                if (freed < need) {
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    bool drained = false;
                    for (;;) {
                        if (!drained) {            // the consumers may be waiting for lines already issued:
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // land all of them first
                            pub = issued * ENG_LINE;
                            if (lane == 0) eng_st_asm(lds0 + L_CTL + C_LANDED * 4, pub);
                            drained = true;
                        }
                        if (__builtin_amdgcn_readfirstlane(eng_ld_asm(lds0 + L_CTL + C_ABORT * 4)) != 0u) { ok = false; break; }
                        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                            eng_fail(a, ctl, ENG_E_LOADER);
                            ok = false;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        freed = eng_min_prog(lds0 + L_CTL + C_PROG * 4);
                        if (freed >= need) break;
                    }
                    ring_wait += __builtin_amdgcn_s_memrealtime() - t0;
                    if (!ok) break;
                }
            }
            for (uint32_t k = 0; k < gn; k++) {
                const uint32_t s0 = (g0 + k) * ENG_LINE;
                if (s0 >= uend_b) {                // next unit (units start at line boundaries, >= 1 line)
                    const EngUnit U = Un;
                    if (++ui < uend_i) Un = ld_unit(a.units, ui);
                    usoff = U.soff;
                    uend_b = usoff + ((U.bytes + ENG_LINE - 1) & ~(ENG_LINE - 1));
                    // a buffer descriptor over the unit's bytes: the lanes of its last line past its end read nothing
                    urs = make_rsrc(reinterpret_cast<const void *>((uint64_t)U.src_lo | (uint64_t)U.src_hi << 32), U.bytes);
                }
                __builtin_amdgcn_raw_ptr_buffer_load_lds(urs, (lds_void_t *)((char *)elds + (s0 & (ENG_RING - 1))), 16,
                                                         s0 - usoff + 16u * (uint32_t)lane, 0, 0, 0);
            }
            issued += gn;
            if (ENG_THIN && __builtin_amdgcn_readfirstlane(eng_ld_asm(lds0 + L_CTL + C_GATHER * 4)) != 0u) {
                // the CU sweeps granules: few lines in flight, so the sweep's loads do not queue behind the stream
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ENG_THIN) : "memory");
                const uint32_t l = issued > (uint32_t)ENG_THIN ? (issued - ENG_THIN) * ENG_LINE : 0u;
                if (l > pub) {
                    pub = l;
                    if (lane == 0) eng_st_asm(lds0 + L_CTL + C_LANDED * 4, pub);
                }
            } else if (issued > (uint32_t)ENG_D) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ENG_D) : "memory");
                const uint32_t l = (issued - ENG_D) * ENG_LINE;
                if (l > pub) {
                    pub = l;
                    if (lane == 0) eng_st_asm(lds0 + L_CTL + C_LANDED * 4, pub);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA may outlive the workgroup
        if (lane == 0) eng_st_asm(lds0 + L_CTL + C_LANDED * 4, ok ? 0xFFFFFFFFu : 0u);
        if (st && lane == 0) {                  // loader start, end, ticks waiting for ring space
            st[0] = tl0;
            st[1] = __builtin_amdgcn_s_memrealtime();
            st[2] = ring_wait;
        }
    } else {
        // ---------------- consumers
        uint32_t ui = cu.unit0;
        const uint32_t uend = cu.unit0 + cu.nunits;
        uint32_t ntask = 0;
        bool abort = false;
        uint32_t *xq = ring + L_XQ / 4;
        float *xd = reinterpret_cast<float *>(ring + L_XD / 4);
        int *xs = reinterpret_cast<int *>(ring + L_XS / 4);
        while (ui < uend && !abort) {
            const uint32_t task = ld_unit(a.units, ui).tmn & 0xFFFFu;
            const EngTask tk = ld_task(a.tasks, task);
            ntask++;
            uint64_t *sk = st && ntask <= (uint32_t)ENG_ST_TASKS ? st + ENG_ST_HDR + ENG_ST_W * (ntask - 1) : nullptr;
            if (w == 0 && sk && lane == 0) {
                sk[0] = __builtin_amdgcn_s_memrealtime();
                sk[3] = task;
            }
            {
                // ---- gather x of this task into LDS, every consumer wave its share (a sweep is one memory round trip
                // queued behind the CU's weight stream, so the waves' shares go in parallel, not in turns); first every
                // wave must have loaded the previous task's x
                if (ENG_THIN && w == 0 && lane == 0) cst(ctl + C_GATHER, 1u);   // the loader thins its stream meanwhile
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (cld(ctl + C_XLOADED) < (uint32_t)ENG_NC * (ntask - 1))
                    if (!eng_spin(a, ctl, t0, ENG_E_XLOADED)) { abort = true; break; }
                if (abort) break;
                const int nb = (int)tk.nb, np = (int)tk.npairs;
                // this wave's items: 8-lane groups of float4 (x from memory) or granules, [i0, i1), in whole 64-lane steps
                const int nitem = nb * 8;
                const int per = ((nitem + 64 * ENG_NC - 1) / (64 * ENG_NC)) * 64;
                const int i0 = w * per, i1 = min(nitem, i0 + per);
                if (tk.xext) {                   // x from memory: the GEMV prologue's quantizer
                    for (int base = i0; base < i1; base += 64) {
                        const int idx = base + lane;                     // float4 index
                        const bool live = idx < i1;
                        const float4 v = live ? reinterpret_cast<const float4 *>(tk.xext)[idx] : make_float4(0, 0, 0, 0);
                        uint32_t d16;
                        int qsum;
                        const uint32_t packed = q8_block_lane(v, d16, qsum);
                        if (live) {
                            const int b = idx >> 3, ww = idx & 7;
                            xq[((((b & 1) << 1) | (ww >> 2)) * np + (b >> 1)) * 4 + (ww & 3)] = packed;
                            if (ww == 0) {
                                xd[b] = h2f(d16);
                                xs[b] = 8 * qsum;
                            }
                        }
                    }
                } else {                         // x from the producers' granules
                    for (int base = i0; base < i1 && !abort; base += 64 * 16) {
                        uint64_t g[16];
                        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
                        for (;;) {
                            bool okl = true;
#pragma unroll
                            for (int k = 0; k < 16; k++) {
                                const int idx = base + lane + 64 * k;
                                g[k] = idx < i1 ? __hip_atomic_load((const g_u64 *)(tk.xgran + idx), __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT)
                                                : (uint64_t)tag << 48;
                                okl &= (uint32_t)(g[k] >> 48) == tag || (a.diag & 1);
                            }
                            if (__builtin_amdgcn_ballot_w64(!okl) == 0) break;   // no lane still waiting
                            if (!eng_spin(a, ctl, t1, ENG_E_GATHER)) { abort = true; break; }
                        }
                        if (abort) break;
#pragma unroll
                        for (int k = 0; k < 16; k++) {
                            const int idx = base + lane + 64 * k;
                            if (idx < i1) {
                                const int b = idx >> 3, ww = idx & 7;
                                xq[((((b & 1) << 1) | (ww >> 2)) * np + (b >> 1)) * 4 + (ww & 3)] = (uint32_t)g[k];
                                const uint32_t aux = (uint32_t)(g[k] >> 32) & 0xFFFFu;
                                if (ww == 0) xd[b] = h2f(aux);
                                if (ww == 1) xs[b] = 8 * (int)(int16_t)aux;
                            }
                        }
                    }
                    if (abort) break;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                // every wave's share in LDS: XGEN counts the waves that finished this task's share
                if (lane == 0) __hip_atomic_fetch_add(ctl + C_XGEN, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
                while (cld(ctl + C_XGEN) < (uint32_t)ENG_NC * ntask)
                    if (!eng_spin(a, ctl, t2, ENG_E_XGEN)) { abort = true; break; }
                if (abort) break;
                if (ENG_THIN && w == 0 && lane == 0) cst(ctl + C_GATHER, 0u);
            }
            asm volatile("" ::: "memory");
            if (w == 0 && sk && lane == 0) sk[1] = __builtin_amdgcn_s_memrealtime();
            const int ppl = ((int)tk.npairs + 63) >> 6;
            if (ppl == 1)
                eng_task_rows<1>(a, ctl, ring, par, tk, ui, uend, task, w, lane, tag, abort, sk);
            else if (ppl == 2)
                eng_task_rows<2>(a, ctl, ring, par, tk, ui, uend, task, w, lane, tag, abort, sk);
            else
                eng_task_rows<3>(a, ctl, ring, par, tk, ui, uend, task, w, lane, tag, abort, sk);
            if (w == 0 && sk && lane == 0) sk[2] = __builtin_amdgcn_s_memrealtime();
        }
        if (lane == 0) cst(ctl + C_PROG + w, 0xFFFFFFFFu);   // never holds the loader back again
    }
    // the last workgroup to finish advances the epoch (every workgroup read it at its start)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const uint64_t old = __hip_atomic_fetch_add(a.ctl + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(a.ctl + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctl + 0, (uint64_t)epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// =============================================================================================== host
struct EnginePlan {
    int device = 0, ncu = 0, ntasks = 0;
    EngTask *d_tasks = nullptr;
    EngUnit *d_units = nullptr;
    EngCU *d_cus = nullptr;
    uint64_t *d_ctl = nullptr;
    uint64_t *d_gran = nullptr;
    uint32_t timeout = 0, diag = 0;
    uint64_t *d_stamps = nullptr;
    size_t units = 0;
    uint64_t max_stream = 0, total_bytes = 0;
};

static void plan_free(EnginePlan *p) {
    if (!p) return;
    if (p->d_tasks) (void)hipFree(p->d_tasks);
    if (p->d_units) (void)hipFree(p->d_units);
    if (p->d_cus) (void)hipFree(p->d_cus);
    if (p->d_ctl) (void)hipFree(p->d_ctl);
    if (p->d_gran) (void)hipFree(p->d_gran);
    if (p->d_stamps) (void)hipFree(p->d_stamps);
    delete p;
}

// The chain shapes the engine takes (else the caller keeps the per-launch chain): every task t >= 1 reads x
// = y[i] of task t - 1 (the same pointer, K <= M_i: its first K values), task 0 reads an x no task writes,
// K <= 12288, outputs of one task disjoint, and every later write of an output region ordered after the
// earlier write by the edges (checked per CU below).
EnginePlan *engine_plan_create(int T, const ggml_hip_chain_task *tk, int ncu, uint32_t timeout_ticks, std::string &why) {
    auto decline = [&](const std::string &m) -> EnginePlan * { why = m; return nullptr; };
    if (T < 1 || T > 65535) return decline("engine: 1..65535 tasks");
    if (ncu < 1 || ncu > 4096) return decline("engine: CU count");
    auto lo = [](const void *p) { return (uint64_t)(uintptr_t)p; };
    std::vector<int> consumed(T, -1);
    for (int t = 0; t < T; t++) {
        const auto &k = tk[t];
        if (k.K > 64 * 3 * 64 || k.K % 64 != 0) return decline("engine: K > 12288");
        for (int i = 0; i < k.nmat; i++) {
            if (k.M[i] >= (1ll << 26)) return decline("engine: M too large");
            for (int j = 0; j < i; j++)
                if (lo(k.y[i]) < lo(k.y[j]) + 4 * (uint64_t)k.M[j] && lo(k.y[j]) < lo(k.y[i]) + 4 * (uint64_t)k.M[i])
                    return decline("engine: sibling outputs overlap");
        }
        if (t == 0) {
            for (int s = 0; s < T; s++)
                for (int i = 0; i < tk[s].nmat; i++)
                    if (lo(k.x) < lo(tk[s].y[i]) + 4 * (uint64_t)tk[s].M[i] && lo(tk[s].y[i]) < lo(k.x) + 4 * (uint64_t)k.K)
                        return decline("engine: the first task's x is written by the chain");
        } else {
            const auto &p = tk[t - 1];
            for (int i = 0; i < p.nmat && consumed[t - 1] < 0; i++)
                if (p.y[i] == k.x && p.M[i] >= k.K) consumed[t - 1] = i;
            if (consumed[t - 1] < 0) return decline("engine: task " + std::to_string(t) + "'s x is not an output of task " +
                                                    std::to_string(t - 1));
        }
    }
    // ---- units, dealt in task order to the least-loaded CU; the consumed output's units first
    struct HU {
        int task, mat, row0, nrows, cu;
        bool consumed, gating;
    };
    std::vector<HU> hu;
    std::vector<std::vector<int>> cu_units(ncu);
    std::vector<uint64_t> load(ncu, 0);
    typedef std::pair<uint64_t, int> LI;
    std::priority_queue<LI, std::vector<LI>, std::greater<LI>> heap;
    for (int c = 0; c < ncu; c++) heap.push(LI(0, c));
    for (int t = 0; t < T; t++) {
        const auto &k = tk[t];
        const uint32_t rowbytes = (uint32_t)(k.K / 64) * 36u;
        std::vector<int> order;
        if (consumed[t] >= 0) order.push_back(consumed[t]);
        for (int i = 0; i < k.nmat; i++)
            if (i != consumed[t]) order.push_back(i);
        for (int i : order) {
            for (int64_t r = 0; r < k.M[i]; r += 32) {
                HU u;
                u.task = t;
                u.mat = i;
                u.row0 = (int)r;
                u.nrows = (int)std::min<int64_t>(32, k.M[i] - r);
                u.consumed = i == consumed[t] && u.nrows == 32;
                u.gating = u.consumed && r < tk[t + 1 < T ? t + 1 : t].K && t + 1 < T;
                const uint64_t bytes = ((uint64_t)u.nrows * rowbytes + ENG_LINE - 1) / ENG_LINE * ENG_LINE;
                LI top = heap.top();
                heap.pop();
                u.cu = top.second;
                top.first += bytes;
                heap.push(top);
                load[u.cu] += bytes;
                cu_units[u.cu].push_back((int)hu.size());
                hu.push_back(u);
            }
        }
    }
    // ---- write-after-write order: an output region written again by a later task t must have every unit of
    // the earlier writer s complete before any unit of t starts.  Units of task u >= 1 start only after every
    // gating unit of task u - 1 finished, and a CU runs its units in order, so it suffices that each CU holding
    // a unit of s has a gating unit in a task in (s, t) (or that unit is gating itself).
    {
        std::vector<std::vector<int>> gates(ncu);       // tasks with gating units, ascending, per CU
        for (int c = 0; c < ncu; c++)
            for (int ix : cu_units[c])
                if (hu[ix].gating && (gates[c].empty() || gates[c].back() != hu[ix].task)) gates[c].push_back(hu[ix].task);
        std::vector<std::vector<std::vector<int>>> cus_of(T);   // [task][mat] -> CUs with a non-gating unit
        for (int t = 0; t < T; t++) cus_of[t].resize(tk[t].nmat);
        for (const HU &u : hu)
            if (!u.gating) cus_of[u.task][u.mat].push_back(u.cu);
        for (int t = 1; t < T; t++)
            for (int j = 0; j < tk[t].nmat; j++) {
                const uint64_t a0 = lo(tk[t].y[j]), a1 = a0 + 4 * (uint64_t)tk[t].M[j];
                bool covered = false;
                for (int s = t - 1; s >= 0 && !covered; s--)
                    for (int i = 0; i < tk[s].nmat; i++) {
                        const uint64_t b0 = lo(tk[s].y[i]), b1 = b0 + 4 * (uint64_t)tk[s].M[i];
                        if (!(a0 < b1 && b0 < a1)) continue;
                        for (int c : cus_of[s][i]) {
                            const auto &g = gates[c];
                            const auto it = std::upper_bound(g.begin(), g.end(), s);
                            if (it == g.end() || *it >= t)
                                return decline("engine: output of task " + std::to_string(t) + " rewrites task " +
                                               std::to_string(s) + "'s without an edge in between on CU " +
                                               std::to_string(c));
                        }
                        if (b0 <= a0 && a1 <= b1) covered = true;   // earlier writers are ordered before s
                    }
            }
    }
    // ---- device tables
    std::vector<EngTask> ht(T);
    std::vector<uint64_t> gran_off(T, ~0ull);
    uint64_t ngran = 0;
    for (int t = 0; t < T; t++)
        if (consumed[t] >= 0) {
            gran_off[t] = ngran;
            ngran += (uint64_t)(tk[t].M[consumed[t]] / 32) * 8;
        }
    auto *p = new EnginePlan;
    p->ncu = ncu;
    p->ntasks = T;
    p->timeout = timeout_ticks;
    hipError_t e = hipSuccess;
    if (ngran) e = hipMalloc(&p->d_gran, ngran * 8);
    if (e == hipSuccess && ngran) e = hipMemset(p->d_gran, 0, ngran * 8);
    for (int t = 0; t < T && e == hipSuccess; t++) {
        const auto &k = tk[t];
        EngTask &d = ht[t];
        memset(&d, 0, sizeof d);
        d.K = (uint32_t)k.K;
        d.nb = (uint32_t)(k.K / 32);
        d.npairs = d.nb / 2;
        d.rowbytes = d.npairs * 36u;
        for (int i = 0; i < k.nmat; i++) d.y[i] = k.y[i];
        if (t == 0) d.xext = k.x;
        else d.xgran = p->d_gran + gran_off[t - 1];
        if (consumed[t] >= 0) d.gran[consumed[t]] = p->d_gran + gran_off[t];
    }
    std::vector<EngUnit> hus;
    std::vector<EngCU> hc(ncu);
    for (int c = 0; c < ncu; c++) {
        hc[c].unit0 = (uint32_t)hus.size();
        hc[c].nunits = (uint32_t)cu_units[c].size();
        uint64_t soff = 0, rbase = 0;
        uint32_t cidx = 0;
        for (int ix : cu_units[c]) {
            const HU &u = hu[ix];
            const auto &k = tk[u.task];
            const uint32_t rowbytes = (uint32_t)(k.K / 64) * 36u;
            EngUnit d;
            const uint64_t src = lo(k.W[u.mat]) + (uint64_t)u.row0 * rowbytes;
            d.src_lo = (uint32_t)src;
            d.src_hi = (uint32_t)(src >> 32);
            d.soff = (uint32_t)soff;
            d.bytes = (uint32_t)u.nrows * rowbytes;
            d.row0 = (uint32_t)u.row0;
            d.rbase = (uint32_t)rbase;
            d.cidx = u.consumed ? cidx++ : ~0u;
            d.tmn = (uint32_t)u.task | (uint32_t)u.mat << 16 | (uint32_t)u.nrows << 24;
            hus.push_back(d);
            soff += ((uint64_t)d.bytes + ENG_LINE - 1) / ENG_LINE * ENG_LINE;
            rbase += (uint64_t)u.nrows;
            p->total_bytes += d.bytes;
        }
        if (soff >= (1ull << 32) - 2 * ENG_RING) {
            plan_free(p);
            return decline("engine: a CU's stream exceeds 4 GiB");
        }
        hc[c].stream_bytes = (uint32_t)soff;
        p->max_stream = std::max<uint64_t>(p->max_stream, soff);
    }
    p->units = hus.size();
    if (e == hipSuccess) e = hipMalloc(&p->d_tasks, sizeof(EngTask) * T);
    if (e == hipSuccess) e = hipMalloc(&p->d_units, sizeof(EngUnit) * std::max<size_t>(1, hus.size()));
    if (e == hipSuccess) e = hipMalloc(&p->d_cus, sizeof(EngCU) * ncu);
    if (e == hipSuccess) e = hipMalloc(&p->d_ctl, 64);
    if (e == hipSuccess) e = hipMemcpy(p->d_tasks, ht.data(), sizeof(EngTask) * T, hipMemcpyHostToDevice);
    if (e == hipSuccess && !hus.empty()) e = hipMemcpy(p->d_units, hus.data(), sizeof(EngUnit) * hus.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_cus, hc.data(), sizeof(EngCU) * ncu, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(p->d_ctl, 0, 64);
    if (e != hipSuccess) {
        plan_free(p);
        return decline(std::string("engine: ") + hipGetErrorString(e));
    }
    if (const char *d = getenv("GGML_HIP_ENGINE_DIAG")) p->diag = (uint32_t)atoi(d);
    if (getenv("GGML_HIP_ENGINE_STAMPS") && atoi(getenv("GGML_HIP_ENGINE_STAMPS")) == 1) {
        const size_t n = (size_t)ncu * ENG_ST_CU * 8;
        if (hipMalloc(&p->d_stamps, n) != hipSuccess || hipMemset(p->d_stamps, 0, n) != hipSuccess) p->d_stamps = nullptr;
    }
    (void)hipGetDevice(&p->device);
    return p;
}

// diagnostics: the stamps of the last launch (GGML_HIP_ENGINE_STAMPS=1 at plan creation), zeroed after the copy
int engine_stamps(EnginePlan *p, uint64_t *out, int64_t n) {
    if (!p->d_stamps) return -1;
    const int64_t need = (int64_t)p->ncu * ENG_ST_CU;
    if (n < need) return (int)need;
    if (hipMemcpy(out, p->d_stamps, need * 8, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    if (hipMemset(p->d_stamps, 0, need * 8) != hipSuccess) return -2;
    return (int)need;
}

hipError_t engine_launch(EnginePlan *p, hipStream_t s) {
    static std::atomic<uint32_t> attr{0};          // one bit per device (16 max)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev > 15) dev = 0;
    if (!(attr.load(std::memory_order_acquire) & (1u << dev))) {
        const hipError_t e = hipFuncSetAttribute((const void *)k_engine_q4_0, hipFuncAttributeMaxDynamicSharedMemorySize, ENG_LDS);
        if (e != hipSuccess) return e;
        attr.fetch_or(1u << dev, std::memory_order_acq_rel);
    }
    EngArgs a;
    a.tasks = p->d_tasks;
    a.units = p->d_units;
    a.cus = p->d_cus;
    a.ctl = p->d_ctl;
    a.timeout = p->timeout;
    a.diag = p->diag;
    a.stamps = p->d_stamps;
    (void)hipGetLastError();
    launch_k(k_engine_q4_0, dim3((unsigned)p->ncu), dim3(ENG_THREADS), ENG_LDS, s, a);
    return hipGetLastError();
}

// error bits of the launches so far (the caller synchronized); detail = the first error's CU << 8 | code
int engine_status(EnginePlan *p, uint64_t *detail) {
    uint64_t c[4] = {0, 0, 0, 0};
    if (hipMemcpy(c, p->d_ctl, 32, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (detail) *detail = c[3];
    return (int)c[2];
}

void engine_plan_destroy(EnginePlan *p) { plan_free(p); }

void engine_plan_info(const EnginePlan *p, int64_t *info) {   // units, max stream bytes per CU, total bytes, CUs
    info[0] = (int64_t)p->units;
    info[1] = (int64_t)p->max_stream;
    info[2] = (int64_t)p->total_bytes;
    info[3] = p->ncu;
}

}  // namespace ghip
