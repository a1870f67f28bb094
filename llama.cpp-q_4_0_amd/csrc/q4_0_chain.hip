// q4_0_chain.hip — a chain of dependent decode (N = 1) q4_0 mul_mats as ONE persistent launch.
//
// What it restates: the sequence of ggml_compute_forward_mul_mat_q_f32 calls (ggml.c:11226-11411)
// that a decode eval issues one after another, each INIT (quantize_row_q8_0 of src1, ggml.c:
// 1192-1275) + COMPUTE (ggml_vec_dot_q4_0_q8_0 per row, ggml.c:2339-2607), with stream order
// between them: task t reads its activation x_t only after every task < t has written its y.
// The per-task arithmetic is the decode GEMV's (q4_0_kernels.hip, k_gemv_q4_0 with row items), so
// every y is bitwise equal to the one-launch-per-mul_mat path — except for a launch the per-launch
// GEMV runs chunk-balanced (BAL: K > 12288 with a row tail, e.g. Falcon's 18176 -> 4544), which sums
// a row's 64-pair chunks separately; the chain keeps the per-lane row order (same oracle bound).
//
// Why one launch: a decode mul_mat streams 9-51 MB of weights in 2-8 us, and each launch pays a
// kernel boundary (~1.5 us) plus a ramp in which the x prologue gates the first rows.  The WEIGHTS
// of task t+1 do not depend on task t, only its x does.  Here every compute wave keeps DEPTH
// weight chunks in flight across task boundaries (a register ring that runs straight from one
// task's rows into the next task's), so HBM streams through the dependency wait.
//
// Roles (one 16-wave workgroup per CU, every workgroup resident; grid = CU count):
//   waves 0..3  control: q8_0-quantize x_t into LDS; publish the workgroup's y rows of task t
//               (write-through sc1 stores, drained) and arrive on a per-XCD counter; poll the
//               counters until every workgroup has finished task t; agent-scope acquire.  They
//               never issue weight loads, so their vmcnt drains wait for nothing else.
//   waves 4..15 compute: rows r = wg + G*j of task t (G = grid), round j on compute slot
//               (j + t) % 12; each row is ceil(K/2048) chunks of 64 block pairs (lane p owns pair
//               64c + p); DEPTH chunks in flight.  A finished row's sum goes to an LDS staging
//               slot (not to global memory: a global store would put a vmcnt drain behind the
//               ring's loads).
// Per task t, every wave passes the same workgroup barriers: A_t (compute done, staging full),
// P_t (counters show task t complete everywhere; acquire done), B_t+1 (x_t+1 in LDS).
// Hand-off protocol: MI355X guide, Guideline 16 (R1 payload stores + counter; relaxed poll,
// one acquire).  Every spin is bounded; a timeout sets sync[8] and the launch drains.
#include "q4_0_kernels.h"

namespace ghip {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) float gfloat;

constexpr int QK = 32;
constexpr int CH_WAVES = 16, CH_NCW = 4, CH_NCOMP = CH_WAVES - CH_NCW;
constexpr int CH_XLOADS = 12;          // float4 x loads in flight per control thread (K <= 12288 in one batch)
constexpr int RSRC_FLAGS = 0x00020000;

__device__ __forceinline__ float h2f(uint32_t bits) {
    _Float16 h;
    const uint16_t b = (uint16_t)bits;
    __builtin_memcpy(&h, &b, 2);
    return (float)h;
}
__device__ __forceinline__ uint32_t f2h(float f) {
    asm volatile("" : "+v"(f));          // see q4_0_kernels.hip: keeps fp16(-0.0) = 0x8000
    const _Float16 h = (_Float16)f;
    uint16_t b;
    __builtin_memcpy(&b, &h, 2);
    return b;
}
__device__ __forceinline__ int q8_round_sat(float v) {
    const float r = __builtin_rintf(v);
    int i = (r >= -2147483648.0f && r < 2147483648.0f) ? (int)r : INT32_MIN;
    i = i > 127 ? 127 : i;
    return i < -128 ? -128 : i;
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float group8_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    return fmaxf(v, dpp_f<0x141>(v));
}
__device__ __forceinline__ int group8_sum(int v) {
    v += dpp_i<0xB1>(v);
    v += dpp_i<0x4E>(v);
    return v + dpp_i<0x141>(v);
}
// same reduction tree as the GEMV (bitwise-equal row sums); total valid in lane 63
__device__ __forceinline__ float wave_sum_lane63(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    v += dpp_f<0x142, 0xA>(v);
    v += dpp_f<0x143, 0xC>(v);
    return v;
}
// quantize_row_q8_0, AVX2 branch (ggml.c:1192-1275), one block over 8 lanes (as q8_block_lane)
__device__ __forceinline__ uint32_t q8_lane(float4 v, uint32_t &d16, int &qsum) {
    float a = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    a = group8_max(a);
    const float d = a / 127.f;
    const float id = (a != 0.0f) ? 127.f / a : 0.0f;
    d16 = f2h(d);
    const int q0 = q8_round_sat(v.x * id), q1 = q8_round_sat(v.y * id);
    const int q2 = q8_round_sat(v.z * id), q3 = q8_round_sat(v.w * id);
    qsum = group8_sum(q0 + q1 + q2 + q3);
    return (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
           ((uint32_t)(q3 & 0xFF) << 24);
}
__device__ __forceinline__ int dot_q4_q8(uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3, const u32x4 xl,
                                         const u32x4 xh) {
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

struct Pair {
    u32x4 a, b;
    uint32_t c;
};

// LDS image of one task (32 words), copied from the device task table at launch
enum : int {
    TW_W = 0,        // 4 x u64 weight bases
    TW_Y = 8,        // 4 x u64 outputs
    TW_X = 16,       // u64 x
    TW_RB = 18,      // row_begin[1..3] (row_begin[0] = 0)
    TW_M = 21,       // total rows (= row_begin[n])
    TW_K = 22,
    TW_WORDS = 32
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// wave-uniform cursor over this compute wave's (task, round, chunk) items
struct Cursor {
    int t, j, c;            // task, round (row = wg + G*j), chunk within the row
    int M, nchunk, npairs;  // of task t
    int rb1, rb2, rb3;
    uint64_t w0, w1, w2, w3;
    int64_t rowbytes;
};

}  // namespace

template <int DEPTH>
__global__ __launch_bounds__(CH_WAVES * 64) void k_gemv_chain_q4_0(const ChainTaskDev *__restrict__ tasks, int ntasks,
                                                                  uint32_t *sync, int spin_limit, int kmax,
                                                                  unsigned long long *stamps) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t *tbl = lds;                                              // [ntasks][32]
    uint32_t *xq = lds + ntasks * TW_WORDS;                           // [4][npairs][4] int8x4
    const int nbmax = kmax / QK;
    float *xd = reinterpret_cast<float *>(xq + nbmax * 8);           // [nb]
    int *xs = reinterpret_cast<int *>(xd + nbmax);                    // [nb] 8*sum(q)
    float *stg = reinterpret_cast<float *>(xs + nbmax);              // [CHAIN_STAGE_MAX] row sums
    __shared__ int s_abort;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = (int)uni((uint32_t)(tid >> 6));
    const int wg = blockIdx.x, G = gridDim.x;
    gu32 *gsync = (gu32 *)(sync);
    // diagnostics (GGML_HIP_CHAIN_STAMPS=1): per (workgroup, task) s_memrealtime at 8 points
#define CHAIN_STAMP(t_, k_)                                                                        \
    do {                                                                                           \
        if (stamps && lane == 0)                                                                   \
            stamps[((size_t)wg * ntasks + (t_)) * 8 + (k_)] = __builtin_amdgcn_s_memrealtime();    \
    } while (0)

    // task table -> LDS (every thread a word), abort flag
    for (int i = tid; i < ntasks * TW_WORDS; i += CH_WAVES * 64)
        tbl[i] = reinterpret_cast<const uint32_t *>(tasks)[i];
    if (tid == 0) s_abort = 0;
    __syncthreads();

    auto tw = [&](int t, int w) __attribute__((always_inline)) { return uni(tbl[t * TW_WORDS + w]); };
    auto tw64 = [&](int t, int w) __attribute__((always_inline)) {
        return (uint64_t)tw(t, w) | ((uint64_t)tw(t, w + 1) << 32);
    };

    // ---- control: quantize x of task t into LDS (bit-exact quantize_row_q8_0) --------------------
    auto load_x = [&](int t) __attribute__((always_inline)) {
        const int K = tw(t, TW_K), nb = K / QK, npairs = nb >> 1, total = nb * 8;
        const float *x = reinterpret_cast<const float *>(tw64(t, TW_X));
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), 0, total * 16, RSRC_FLAGS);
        for (int base = 0; base < total; base += CH_XLOADS * CH_NCW * 64) {
            u32x4 xv[CH_XLOADS];
#pragma unroll
            for (int i = 0; i < CH_XLOADS; i++)
                // sc1 (agent-coherent) loads: every handed-off byte was stored sc1 and drained before
                // its arrival, so no acquire fence is needed (MI355X guide, Guideline 16 Rule)
                xv[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * CH_NCW * 64), 0, 16);
#pragma unroll
            for (int i = 0; i < CH_XLOADS; i++) {
                const int tt = base + tid + i * CH_NCW * 64;
                if (tt < total) {                                     // whole 8-lane groups agree
                    const float4 v = make_float4(__uint_as_float(xv[i].x), __uint_as_float(xv[i].y),
                                                 __uint_as_float(xv[i].z), __uint_as_float(xv[i].w));
                    uint32_t d16;
                    int qsum;
                    const uint32_t packed = q8_lane(v, d16, qsum);
                    const int b = tt >> 3, w = tt & 7;
                    xq[((((b & 1) << 1) | (w >> 2)) * npairs + (b >> 1)) * 4 + (w & 3)] = packed;
                    if ((tt & 7) == 0) {
                        xd[b] = h2f(d16);
                        xs[b] = 8 * qsum;
                    }
                }
            }
        }
    };

    if (wave < CH_NCW) {
        // ======================= control waves =======================
        load_x(0);
        __syncthreads();                                              // B_0
        const int xcd = wg & 7;                                       // counter shard (speed only)
        const uint32_t nx = (uint32_t)(G / 8 + (xcd < G % 8 ? 1 : 0));  // workgroups on this shard
        const uint32_t nshard = (uint32_t)(G < 8 ? G : 8);
        for (int t = 0; t < ntasks; t++) {
            __syncthreads();                                          // A_t: staging of task t full
            if (wave == 0) {
                CHAIN_STAMP(t, 0);
                const int M = tw(t, TW_M);
                const int rb1 = tw(t, TW_RB), rb2 = tw(t, TW_RB + 1), rb3 = tw(t, TW_RB + 2);
                const uint64_t y0 = tw64(t, TW_Y), y1 = tw64(t, TW_Y + 2), y2 = tw64(t, TW_Y + 4),
                               y3 = tw64(t, TW_Y + 6);
                const int nrounds = wg < M ? (M - 1 - wg) / G + 1 : 0;
                for (int j = lane; j < nrounds; j += 64) {
                    const int r = wg + G * j;
                    const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
                    // delta selects (a ternary chain over four values becomes a scratch lookup table)
                    const uint64_t yb = y0 + (g1 ? y1 - y0 : 0) + (g2 ? y2 - y1 : 0) + (g3 ? y3 - y2 : 0);
                    const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
                    // R1 payload store: write-through (sc1), no release fence needed
                    __hip_atomic_store((gfloat *)(yb) + (r - rb), stg[j], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the y stores have completed
                // two-level arrival: the shard's last arriver of task t adds to the top counter
                if (lane == 0) {
                    const uint32_t old = __hip_atomic_fetch_add(gsync + CHAIN_SHARD_STRIDE * (1 + xcd), 1u,
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (old + 1 == (uint32_t)(t + 1) * nx)
                        __hip_atomic_fetch_add(gsync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                CHAIN_STAMP(t, 1);
                if (t + 1 < ntasks && !s_abort) {
                    // poll: every XCD counter has (t+1) arrivals per workgroup of that XCD
                    // poll the top counter: every shard's last arriver has added (t+1) times
                    const uint32_t target = (uint32_t)(t + 1) * nshard;
                    int spins = 0;
                    for (;;) {
                        const uint32_t v = uni(__hip_atomic_load(gsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        if (v >= target) break;
                        if (++spins > spin_limit) {
                            if (lane == 0) {
                                __hip_atomic_store(gsync + CHAIN_SHARD_STRIDE * 9, (uint32_t)(t + 1), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                                s_abort = 1;
                            }
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    CHAIN_STAMP(t, 2);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler ordering only
                    CHAIN_STAMP(t, 3);
                }
            }
            if (t + 1 < ntasks) {
                __syncthreads();                                      // P_t: task t complete everywhere
                load_x(t + 1);
                if (wave == 0) CHAIN_STAMP(t, 4);
                __syncthreads();                                      // B_t+1: x_t+1 in LDS
            }
        }
        return;
    }

    // ========================= compute waves =========================
    const int slot = wave - CH_NCW;
    auto load_task = [&](Cursor &cu, int t) __attribute__((always_inline)) {
        cu.t = t;
        cu.M = tw(t, TW_M);
        const int K = tw(t, TW_K);
        cu.npairs = K / 64;
        cu.nchunk = (cu.npairs + 63) >> 6;
        cu.rowbytes = (int64_t)(K / QK) * 18;
        cu.rb1 = tw(t, TW_RB);
        cu.rb2 = tw(t, TW_RB + 1);
        cu.rb3 = tw(t, TW_RB + 2);
        cu.w0 = tw64(t, TW_W);
        cu.w1 = tw64(t, TW_W + 2);
        cu.w2 = tw64(t, TW_W + 4);
        cu.w3 = tw64(t, TW_W + 6);
    };
    // first item of this wave at or after task t
    auto seek = [&](Cursor &cu, int t) __attribute__((always_inline)) {
        for (; t < ntasks; t++) {
            int j0 = (slot - t) % CH_NCOMP;
            j0 += j0 < 0 ? CH_NCOMP : 0;
            if (wg + G * j0 < tw(t, TW_M)) {
                load_task(cu, t);
                cu.j = j0;
                cu.c = 0;
                return;
            }
        }
        cu.t = ntasks;
    };
    auto advance = [&](Cursor &cu) __attribute__((always_inline)) {
        if (++cu.c < cu.nchunk) return;
        cu.c = 0;
        cu.j += CH_NCOMP;
        if (wg + G * cu.j < cu.M) return;
        seek(cu, cu.t + 1);
    };
    // a dummy in-bounds address for past-the-end ring slots (task 0, row 0, pair 0: no traffic)
    const uint64_t dummy = tw64(0, TW_W);
    auto issue = [&](const Cursor &cu) __attribute__((always_inline)) {
        Pair v;
        const uint8_t *p36;
        if (cu.t < ntasks) {
            const int r = wg + G * cu.j;
            const bool g1 = r >= cu.rb1, g2 = r >= cu.rb2, g3 = r >= cu.rb3;
            const uint64_t wb = cu.w0 + (g1 ? cu.w1 - cu.w0 : 0) + (g2 ? cu.w2 - cu.w1 : 0) + (g3 ? cu.w3 - cu.w2 : 0);
            const int rb = (g1 ? cu.rb1 : 0) + (g2 ? cu.rb2 - cu.rb1 : 0) + (g3 ? cu.rb3 - cu.rb2 : 0);
            const int pp = 64 * cu.c + lane;
            const int pc = pp < cu.npairs ? pp : cu.npairs - 1;
            p36 = reinterpret_cast<const uint8_t *>(wb) + (int64_t)(r - rb) * cu.rowbytes + 36 * pc;
        } else {
            p36 = reinterpret_cast<const uint8_t *>(dummy);
        }
        v.a = *(g_u32x4 *)(p36);
        v.b = *(g_u32x4 *)(p36 + 16);
        v.c = *(g_u32 *)(p36 + 32);
        return v;
    };

    Cursor ic, pc;
    seek(ic, 0);
    pc = ic;
    Pair buf[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
        buf[d] = issue(ic);
        if (ic.t < ntasks) advance(ic);
    }
    __syncthreads();                                                  // B_0
    int tcur = 0;
    float acc = 0.0f;
    auto process = [&](const Pair &v) __attribute__((always_inline)) {
        const int p = 64 * pc.c + lane;
        if (p < pc.npairs) {
            const int np = pc.npairs;
            const float dA = h2f(v.a.x & 0xFFFFu);
            const float dB = h2f(v.b.x >> 16);
            const uint32_t qA0 = __builtin_amdgcn_alignbyte(v.a.y, v.a.x, 2);
            const uint32_t qA1 = __builtin_amdgcn_alignbyte(v.a.z, v.a.y, 2);
            const uint32_t qA2 = __builtin_amdgcn_alignbyte(v.a.w, v.a.z, 2);
            const uint32_t qA3 = __builtin_amdgcn_alignbyte(v.b.x, v.a.w, 2);
            const float2 dx = *reinterpret_cast<const float2 *>(xd + 2 * p);
            const int2 sx = *reinterpret_cast<const int2 *>(xs + 2 * p);
            const u32x4 *xc = reinterpret_cast<const u32x4 *>(xq) + p;
            const int sA = dot_q4_q8(qA0, qA1, qA2, qA3, xc[0], xc[np]) - sx.x;
            const int sB = dot_q4_q8(v.b.y, v.b.z, v.b.w, v.c, xc[2 * np], xc[3 * np]) - sx.y;
            acc = fmaf((float)sA, dA * dx.x, acc);
            acc = fmaf((float)sB, dB * dx.y, acc);
        }
        if (pc.c == pc.nchunk - 1) {                                  // row complete
            const float tsum = wave_sum_lane63(acc);
            if (lane == 63) stg[pc.j] = tsum;
            acc = 0.0f;
        }
    };
    for (;;) {
#pragma unroll
        for (int d = 0; d < DEPTH; d++) {
            if (pc.t >= ntasks) goto done;
            while (tcur < pc.t) {                                     // leave task tcur: A, P, B
                __syncthreads();
                __syncthreads();
                __syncthreads();
                tcur++;
            }
            if (stamps && slot == 0 && pc.j < CH_NCOMP && pc.c == 0) CHAIN_STAMP(pc.t, 5);
            process(buf[d]);
            if (stamps && slot == 0 && pc.c == pc.nchunk - 1) CHAIN_STAMP(pc.t, 6);
            buf[d] = issue(ic);
            if (ic.t < ntasks) advance(ic);
            advance(pc);
        }
    }
done:
    for (; tcur < ntasks; tcur++) {
        __syncthreads();                                              // A
        if (tcur + 1 < ntasks) {
            __syncthreads();                                          // P
            __syncthreads();                                          // B
        }
    }
}

template <int DEPTH>
static hipError_t launch_chain_d(const ChainTaskDev *tasks, int ntasks, uint32_t *sync, int kmax, int grid,
                                 unsigned long long *stamps, hipStream_t s) {
    const size_t lds = chain_lds_bytes(ntasks, kmax);
    static int spin = 0;
    if (spin == 0) {
        const char *e = getenv("GGML_HIP_CHAIN_SPIN");
        spin = e ? atoi(e) : (1 << 22);
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(k_gemv_chain_q4_0<DEPTH>, dim3(grid), dim3(CH_WAVES * 64), lds, s, tasks, ntasks, sync, spin,
                       kmax, stamps);
    return hipGetLastError();
}

size_t chain_lds_bytes(int ntasks, int kmax) {
    return (size_t)ntasks * TW_WORDS * 4 + (size_t)(kmax / QK) * 40 + CHAIN_STAGE_MAX * 4;
}

int chain_max_workgroups(int kmax, int ntasks, int depth) {
    int occ = 0;
    const size_t lds = chain_lds_bytes(ntasks, kmax);
    hipError_t e;
    switch (depth) {
        case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gemv_chain_q4_0<2>, CH_WAVES * 64, lds); break;
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gemv_chain_q4_0<4>, CH_WAVES * 64, lds); break;
        case 6: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gemv_chain_q4_0<6>, CH_WAVES * 64, lds); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gemv_chain_q4_0<8>, CH_WAVES * 64, lds); break;
    }
    return e == hipSuccess ? occ : 0;
}

hipError_t gemv_chain_q4_0(const ChainTaskDev *tasks, int ntasks, uint32_t *sync, int kmax, int grid, int depth,
                           unsigned long long *stamps, hipStream_t s) {
    switch (depth) {
        case 2: return launch_chain_d<2>(tasks, ntasks, sync, kmax, grid, stamps, s);
        case 4: return launch_chain_d<4>(tasks, ntasks, sync, kmax, grid, stamps, s);
        case 6: return launch_chain_d<6>(tasks, ntasks, sync, kmax, grid, stamps, s);
        default: return launch_chain_d<8>(tasks, ntasks, sync, kmax, grid, stamps, s);
    }
}

}  // namespace ghip
