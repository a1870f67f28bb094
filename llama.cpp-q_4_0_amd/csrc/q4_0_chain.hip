// q4_0_chain.hip — a chain of dependent decode (N = 1) q4_0 mul_mats as overlapped launches.
//
// What it restates: the sequence of ggml_compute_forward_mul_mat_q_f32 calls (ggml.c:11226-11411)
// that a decode eval issues one after another, each INIT (quantize_row_q8_0 of src1, ggml.c:
// 1192-1275) + COMPUTE (ggml_vec_dot_q4_0_q8_0 per row, ggml.c:2339-2607), with stream order
// between them: task t reads its activation x_t only after every task < t has written its y.
// The per-row arithmetic is the decode GEMV's (q4_0_kernels.hip, k_gemv_q4_0 with row items: the
// same per-lane fma order and the same DPP reduction), so every y is bitwise equal to the
// one-launch-per-mul_mat path — except where that path runs chunk-balanced (BAL: K > 12288 with a
// row tail), which sums a row's 64-pair chunks separately (same oracle bound).
//
// Why: a decode mul_mat streams 9-51 MB of weights in 2-8 us, and one launch after another pays a
// kernel boundary plus a ramp in which nothing streams (~2.8 us fixed per launch).
// The WEIGHTS of task t do not depend on task t-1, only its x does.  So task t is its own launch on
// the other of two streams: it becomes resident while task t-1 still runs (each launch is one
// 8-wave workgroup per CU at <= 128 VGPRs, half a CU, so two consecutive launches always fit side
// by side), issues the loads of ALL its rows into a register ring (up to ~150 KB per CU, the whole
// matrix for most LLaMA shapes), and only then waits for task t-1's workgroups to have published
// their y.  Stream order (t-2 -> t on one stream) keeps at most two launches in flight, which is
// what makes the co-residency argument hold: a waiting launch can never keep its producer from
// being dispatched.
//
// Hand-off (MI355X_MICROARCH.md, "Valid forms", table row 1): every storing wave writes its y with
// sc1 (write-through) stores and drains them (s_waitcnt vmcnt(0)); after a workgroup barrier one
// lane stores the workgroup's flag (sc1) = the chain's epoch.  The consumer's wave 0 polls the
// producer's flags with sc1 loads; the workgroup's other waves join a barrier behind it, and every
// load of x is an sc1 load.  The epoch is bumped by a one-thread kernel at the start of every chain
// launch (a kernel boundary before the first task), so no flag is ever reset and a replayed graph
// needs no memset.  Every wait is bounded: a timeout records the task in the error word (read by
// ggml_hip_chain_status) and the launch drains.
#include "q4_0_kernels.h"

#include <climits>

namespace ghip {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) float gfloat;

constexpr int QK = 32;
constexpr int OV_WAVES = 8, OV_THREADS = OV_WAVES * 64;
constexpr int RSRC_FLAGS = 0x00020000;
constexpr int AUX_SC1 = 16;            // buffer-load cache policy: sc1 (agent-coherent, bypasses L1)

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
// the GEMV's reduction tree (bitwise-equal row sums); total valid in lane 63
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

}  // namespace

// One task of the chain (kernel argument, by value).
struct OvlArgs {
    const uint8_t *W[4];
    float *y[4];
    int rb1, rb2, rb3, M;       // row_begin[1..3] of the concatenated sibling rows, total rows
    int nb;                     // K / 32
    int task;                   // index + 1 reported on a timeout
    const float *x;
    const uint32_t *wait;       // the producer launch's flags (nullptr: first task)
    int nwait;                  // the producer launch's workgroups
    int spin_limit;
    uint32_t *flags;            // this launch's flags [grid]
    const uint32_t *epoch;
    uint32_t *err;
    unsigned long long *stamps;  // diagnostics (GGML_HIP_CHAIN_STAMPS=1): [task][256 WGs][8] s_memrealtime
};

// PPL = block pairs per lane per row (ceil(K / 4096)), RPW = rows per row wave in the register ring.
// 8 waves, at most 128 VGPRs: two such workgroups (two consecutive tasks) fit one CU.
// Roles: waves 0 .. XW-1 (XW = 2..4 by K) are x-waves: wave 0 polls the producer's flags, then the
// x-waves load x (one batch of OV_XL float4 per lane in flight) and quantize it into LDS; they issue
// no weight loads, so nothing of their own queues ahead of the x loads.  Waves XW..7 are row waves:
// they issue their first RPW rows at once and process rows once x is in LDS, refilling the ring.
constexpr int OV_XL = 16;
__device__ __forceinline__ int ovl_xwaves(int nb) { return nb <= 128 ? 2 : nb <= 256 ? 3 : 4; }

template <int PPL, int RPW>
__global__ __launch_bounds__(OV_THREADS, 4) void k_gemv_ovl_q4_0(const OvlArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ int s_go;
    const int nb = a.nb, npairs = nb >> 1;
    uint32_t *xq = lds;                                               // [4][npairs][4] int8x4
    float *xd = reinterpret_cast<float *>(xq + nb * 8);               // [nb]
    int *xs = reinterpret_cast<int *>(xd + nb);                       // [nb] 8*sum(q)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int XW = ovl_xwaves(nb), ROWW = OV_WAVES - XW;
    const bool xwave = wave < XW;
    const int G = gridDim.x, S = G * ROWW;
    const int gw = blockIdx.x * ROWW + (wave - XW);                   // row wave: rows gw, gw + S, ...
    const int M = a.M;
    const int nrows = !xwave && gw < M ? (M - 1 - gw) / S + 1 : 0;    // <= 64 (host check)
    const int64_t rowbytes = (int64_t)nb * 18;
    unsigned long long *const stp = a.stamps ? a.stamps + ((size_t)(a.task - 1) * 256 + blockIdx.x) * 8 : nullptr;
    // stamps 0, 2, 3, 6 by the first x-wave, 1, 4, 5 by the first row wave
#define OVL_STAMP(k_, w_)                                                     \
    do {                                                                      \
        if (stp && tid == 64 * (w_)) stp[k_] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    OVL_STAMP(0, 0);
    if (tid == 0) s_go = 0;

    const uint64_t w0 = (uint64_t)a.W[0], wd1 = (uint64_t)a.W[1] - w0, wd2 = (uint64_t)a.W[2] - (uint64_t)a.W[1],
                   wd3 = (uint64_t)a.W[3] - (uint64_t)a.W[2];
    const int rb1 = a.rb1, rb2 = a.rb2, rb3 = a.rb3;
    // sums of selected deltas: s_cselect / v_cndmask, no scratch lookup table
    auto row_ptr = [&](int r) __attribute__((always_inline)) {
        const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
        const uint64_t w = w0 + (g1 ? wd1 : 0) + (g2 ? wd2 : 0) + (g3 ? wd3 : 0);
        const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
        return reinterpret_cast<const uint8_t *>(w) + (int64_t)(r - rb) * rowbytes;
    };
    struct Row {
        Pair p[PPL];
    };
    // row i of this wave (wave-uniform guard: past the end nothing is loaded)
    auto issue = [&](Row &v, int i) __attribute__((always_inline)) {
        if (i < nrows) {
            const uint8_t *rp = row_ptr(gw + i * S);
#pragma unroll
            for (int j = 0; j < PPL; j++) {
                const int pp = 64 * j + lane;
                const uint8_t *p36 = rp + 36 * (pp < npairs ? pp : npairs - 1);
                v.p[j].a = *(g_u32x4 *)(p36);
                v.p[j].b = *(g_u32x4 *)(p36 + 16);
                v.p[j].c = *(g_u32 *)(p36 + 32);
            }
        }
    };

    Row buf[RPW];
    if (!xwave) {
        // ---- row waves: the ring's rows in flight before the dependency wait
#pragma unroll
        for (int d = 0; d < RPW; d++) issue(buf[d], d);
        OVL_STAMP(1, XW);
    } else {
        // ---- x-waves: wait for the producer (task t-1), wave 0 polls its workgroups' flags (an
        // earlier task's wait already gave up: drain without waiting, the launch's results are invalid)
        if (wave == 0) {
            const uint32_t epoch = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (a.wait && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
                const int nw = a.nwait;
                int spins = 0;
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int i = lane + 64 * k;
                        if (i < nw) ok &= __hip_atomic_load(a.wait + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
                    }
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                    if (++spins > a.spin_limit) {
                        if (lane == 0) __hip_atomic_store(a.err, (uint32_t)a.task, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            OVL_STAMP(2, 0);
            if (lane == 0) __hip_atomic_store(&s_go, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            while (__hip_atomic_load(&s_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                __builtin_amdgcn_s_sleep(1);
        }
        // ---- INIT: q8_0 of x into LDS (bit-exact quantize_row_q8_0), sc1 loads of the handed-off x
        const int total = nb * 8;                                    // float4 units
        const int XT = XW * 64;
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.x), 0, total * 16, RSRC_FLAGS);
        for (int base = 0; base < total; base += OV_XL * XT) {
            u32x4 xv[OV_XL];
#pragma unroll
            for (int i = 0; i < OV_XL; i++)                              // past the end: 0, no traffic
                xv[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, 16 * (base + tid + i * XT), 0, AUX_SC1);
#pragma unroll
            for (int i = 0; i < OV_XL; i++) {
                const int t = base + tid + i * XT;
                if (t < total) {                                     // whole 8-lane groups agree
                    const float4 v = make_float4(__uint_as_float(xv[i].x), __uint_as_float(xv[i].y),
                                                 __uint_as_float(xv[i].z), __uint_as_float(xv[i].w));
                    uint32_t d16;
                    int qsum;
                    const uint32_t packed = q8_lane(v, d16, qsum);
                    const int b = t >> 3, w = t & 7;
                    xq[((((b & 1) << 1) | (w >> 2)) * npairs + (b >> 1)) * 4 + (w & 3)] = packed;
                    if ((t & 7) == 0) {
                        xd[b] = h2f(d16);
                        xs[b] = 8 * qsum;
                    }
                }
            }
        }
        OVL_STAMP(3, 0);
    }
    __syncthreads();                                                  // x in LDS
    OVL_STAMP(4, XW);

    // ---- COMPUTE (row waves): the GEMV's row-item arithmetic; lane i keeps row i's sum for the store
    float ysum = 0.0f;
    auto process = [&](const Row &v) __attribute__((always_inline)) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < PPL; j++) {
            const Pair &pr = v.p[j];
            const int p = 64 * j + lane;
            if (p < npairs) {
                const float dA = h2f(pr.a.x & 0xFFFFu);
                const float dB = h2f(pr.b.x >> 16);
                const uint32_t qA0 = __builtin_amdgcn_alignbyte(pr.a.y, pr.a.x, 2);
                const uint32_t qA1 = __builtin_amdgcn_alignbyte(pr.a.z, pr.a.y, 2);
                const uint32_t qA2 = __builtin_amdgcn_alignbyte(pr.a.w, pr.a.z, 2);
                const uint32_t qA3 = __builtin_amdgcn_alignbyte(pr.b.x, pr.a.w, 2);
                const float2 dx = *reinterpret_cast<const float2 *>(xd + 2 * p);
                const int2 sx = *reinterpret_cast<const int2 *>(xs + 2 * p);
                const u32x4 *xc = reinterpret_cast<const u32x4 *>(xq) + p;
                const int sA = dot_q4_q8(qA0, qA1, qA2, qA3, xc[0], xc[npairs]) - sx.x;
                const int sB = dot_q4_q8(pr.b.y, pr.b.z, pr.b.w, pr.c, xc[2 * npairs], xc[3 * npairs]) - sx.y;
                acc = fmaf((float)sA, dA * dx.x, acc);
                acc = fmaf((float)sB, dB * dx.y, acc);
            }
            // long rows: keep the scheduler from hoisting every pair's LDS operands (spills at PPL 6)
            if constexpr (PPL > 4) __builtin_amdgcn_sched_barrier(0);
        }
        const float t = wave_sum_lane63(acc);
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 63));
    };
    for (int it = 0; it < nrows; it += RPW) {
#pragma unroll
        for (int d = 0; d < RPW; d++) {
            if (it + d >= nrows) break;
            const float s = process(buf[d]);
            ysum = lane == it + d ? s : ysum;
            issue(buf[d], it + d + RPW);
        }
    }
    OVL_STAMP(5, XW);

    // ---- publish: sc1 stores of the wave's rows, drained, then one flag per workgroup
    if (lane < nrows) {
        const int r = gw + lane * S;
        const bool g1 = r >= rb1, g2 = r >= rb2, g3 = r >= rb3;
        const uint64_t y0 = (uint64_t)a.y[0];
        const uint64_t yb = y0 + (g1 ? (uint64_t)a.y[1] - y0 : 0) + (g2 ? (uint64_t)a.y[2] - (uint64_t)a.y[1] : 0) +
                            (g3 ? (uint64_t)a.y[3] - (uint64_t)a.y[2] : 0);
        const int rb = (g1 ? rb1 : 0) + (g2 ? rb2 - rb1 : 0) + (g3 ? rb3 - rb2 : 0);
        __hip_atomic_store(reinterpret_cast<float *>(yb) + (r - rb), ysum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    OVL_STAMP(6, 0);
    if (tid == 0) {
        const uint32_t epoch = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.flags + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#undef OVL_STAMP
}

__global__ void k_ovl_bump(uint32_t *epoch, uint32_t *err) {
    epoch[0] += 1;
    err[0] = 0;
}

namespace {

template <int PPL>
constexpr int ovl_rpw() {
    // ~70-90 VGPRs of ring, 128 in all without spills (-Rpass-analysis=kernel-resource-usage)
    return PPL == 1 ? 8 : PPL == 2 ? 4 : PPL == 3 ? 3 : PPL == 4 ? 2 : 1;
}

template <int PPL>
const void *ovl_kernel() {
    return reinterpret_cast<const void *>(&k_gemv_ovl_q4_0<PPL, ovl_rpw<PPL>()>);
}

const void *ovl_kernel_ppl(int ppl) {
    switch (ppl) {
        case 1: return ovl_kernel<1>();
        case 2: return ovl_kernel<2>();
        case 3: return ovl_kernel<3>();
        case 4: return ovl_kernel<4>();
        case 5: return ovl_kernel<5>();
        case 6: return ovl_kernel<6>();
        default: return nullptr;
    }
}

}  // namespace

int chain_ovl_rows_per_wave(int64_t K) {
    const int ppl = (int)((K / 64 + 63) / 64);
    switch (ppl) {
        case 1: return ovl_rpw<1>();
        case 2: return ovl_rpw<2>();
        case 3: return ovl_rpw<3>();
        case 4: return ovl_rpw<4>();
        case 5: return ovl_rpw<5>();
        case 6: return ovl_rpw<6>();
        default: return 0;
    }
}

int chain_ovl_occupancy(int64_t K) {
    const void *k = ovl_kernel_ppl((int)((K / 64 + 63) / 64));
    if (!k) return 0;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, OV_THREADS, chain_ovl_lds_bytes(K)) != hipSuccess)
        return 0;
    return occ;
}

size_t chain_ovl_lds_bytes(int64_t K) { return (size_t)(K / QK) * 40; }

int chain_ovl_grid(int64_t M, int num_cus) {
    const int64_t need = (M + OV_WAVES - 1) / OV_WAVES;
    return (int)(need < num_cus ? need : num_cus);
}

hipError_t chain_ovl_bump(uint32_t *epoch, uint32_t *err, hipStream_t s) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(k_ovl_bump, dim3(1), dim3(1), 0, s, epoch, err);
    return hipGetLastError();
}

hipError_t chain_ovl_launch(const ChainOvlTask &t, const uint32_t *wait, int nwait, uint32_t *flags,
                            const uint32_t *epoch, uint32_t *err, int spin_limit, int num_cus, hipStream_t s,
                            unsigned long long *stamps) {
    const int ppl = (int)((t.K / 64 + 63) / 64);
    if (t.K <= 0 || t.K % 64 != 0 || ppl < 1 || ppl > CHAIN_OVL_MAX_PPL) return hipErrorInvalidValue;
    const int grid = chain_ovl_grid(t.M, num_cus);
    if (grid < 1 || (int64_t)grid * (OV_WAVES - 4) * 64 < t.M || t.M > INT_MAX) return hipErrorInvalidValue;
    OvlArgs a;
    for (int i = 0; i < 4; i++) {
        a.W[i] = reinterpret_cast<const uint8_t *>(t.W[i]);
        a.y[i] = t.y[i];
    }
    a.rb1 = t.rb[0];
    a.rb2 = t.rb[1];
    a.rb3 = t.rb[2];
    a.M = (int)t.M;
    a.nb = (int)(t.K / QK);
    a.task = t.index + 1;
    a.x = t.x;
    a.wait = wait;
    a.nwait = nwait;
    a.spin_limit = spin_limit;
    a.flags = flags;
    a.epoch = epoch;
    a.err = err;
    a.stamps = stamps;
    const size_t lds = chain_ovl_lds_bytes(t.K);
    (void)hipGetLastError();
    switch (ppl) {
#define OVL_CASE(P)                                                                                         \
    case P:                                                                                                 \
        hipLaunchKernelGGL((k_gemv_ovl_q4_0<P, ovl_rpw<P>()>), dim3(grid), dim3(OV_THREADS), lds, s, a); \
        break;
        OVL_CASE(1)
        OVL_CASE(2)
        OVL_CASE(3)
        OVL_CASE(4)
        OVL_CASE(5)
        OVL_CASE(6)
#undef OVL_CASE
    }
    return hipGetLastError();
}

}  // namespace ghip
