/*
 * ggml-hip.h — C ABI of the MI355X-native (gfx950) q4_0 mul_mat backend for ggml.
 *
 * Drop-in for the reference's GPU backend ABI, ggml-cuda.h:15-36 of
 * Fcucgvhhhvjv/llama.cpp-q_4_0 (the hook sites in ggml.c / llama.cpp /
 * arch/arch-util.h call these exactly where they call ggml_cuda_*; see
 * INTEGRATION.md).  Plain pointers and sizes only; no torch types.
 *
 * Scope: GGML_OP_MUL_MAT with src0 = GGML_TYPE_Q4_0, src1 = dst = GGML_TYPE_F32
 * (the path BASELINE.json names).  Everything else returns "cannot" so ggml's
 * CPU path runs, exactly as ggml_cuda_can_mul_mat / ggml_cuda_compute_forward
 * return false for what they do not handle.
 *
 * Numerics (pinned by tests/): the q8_0 activation bytes are bit-exact to the
 * AVX2 branch of quantize_row_q8_0 (ggml.c:1192-1275); y agrees with
 * ggml_vec_dot_q4_0_q8_0 within 1e-3 relative + fp32 accumulation bound.
 */
#ifndef GGML_HIP_H
#define GGML_HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_HIP_MAX_DEVICES 16   /* GGML_CUDA_MAX_DEVICES, ggml-cuda.h:9 */

struct ggml_tensor;              /* ggml.h:378-414 (mirrored bit-for-bit in csrc/ggml_abi.h) */
struct ggml_compute_params;      /* ggml.h:459-468 */

/* tensor->extra of device-resident tensors (ggml-cuda.h:11-13): one pointer per
 * device; for GGML_BACKEND_GPU_SPLIT tensors device i holds its row slice. */
struct ggml_tensor_extra_gpu {
    void *data_device[GGML_HIP_MAX_DEVICES];
};

/* status codes of the tensor-free entry points */
enum ggml_hip_status {
    GGML_HIP_OK = 0,
    GGML_HIP_ERR_INVALID = -1,      /* bad shape / pointer / alignment */
    GGML_HIP_ERR_UNSUPPORTED = -2,  /* valid request outside the q4_0 path */
    GGML_HIP_ERR_DEVICE = -3,       /* HIP runtime error (message on stderr) */
    GGML_HIP_ERR_NOMEM = -4,
    GGML_HIP_ERR_COMM = -5,         /* RCCL error */
};

/* ------------------------------------------------------------------------------------------
 * ggml-cuda.h equivalents (same argument meaning, same error behaviour: HIP errors are
 * fatal with a message, like CUDA_CHECK in ggml-cuda.cu:22-51).
 * ---------------------------------------------------------------------------------------- */

/* ggml_init_cublas (ggml-cuda.h:15, ggml-cuda.cu:1826-1861): enumerate devices, default
 * split proportional to VRAM, one non-blocking stream per device.  Idempotent, thread-safe. */
void   ggml_init_hip(void);
/* ggml_cuda_set_tensor_split (ggml-cuda.h:16): per-device fractions (cumulative sums are
 * normalised, all-zero = keep default). */
void   ggml_hip_set_tensor_split(const float *tensor_split);
/* ggml_cuda_can_mul_mat (ggml-cuda.h:19, ggml-cuda.cu:2595-2610). */
bool   ggml_hip_can_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                            struct ggml_tensor *dst);
/* ggml-cuda.h:20 declares ggml_cuda_mul_mat_get_wsize but ggml-cuda.cu never defines it; ours
 * returns 0 (no host work buffer is needed). */
size_t ggml_hip_mul_mat_get_wsize(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                                  struct ggml_tensor *dst);
/* ggml_cuda_mul_mat (ggml-cuda.h:21 / ggml-cuda.cu:2671): dst = src0 x src1 for Q4_0 src0.
 * Operands may be host (GGML_BACKEND_CPU) or device resident; synchronous on return when dst
 * is a host tensor. */
void   ggml_hip_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                        struct ggml_tensor *dst);
/* ggml_cuda_mul (ggml-cuda.h:18, ggml-cuda.cu:2580-2583): dst = src0 * src1 (F32, src1 rows
 * repeated over src0), on the device, operands host or device resident. */
void   ggml_hip_mul(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst);
/* ggml_cuda_host_malloc / host_free (ggml-cuda.h:24-25): pinned host memory, NULL on failure. */
void  *ggml_hip_host_malloc(size_t size);
void   ggml_hip_host_free(void *ptr);
/* ggml_cuda_transform_tensor (ggml-cuda.h:27, ggml-cuda.cu:2766-2809): upload tensor data
 * (whole, or the device's row slice for GGML_BACKEND_GPU_SPLIT) and set tensor->extra. */
void   ggml_hip_transform_tensor(void *data, struct ggml_tensor *tensor);
/* ggml_cuda_free_data (ggml-cuda.h:29). */
void   ggml_hip_free_data(struct ggml_tensor *tensor);
/* ggml_cuda_assign_buffers{,_no_scratch,_force_inplace} (ggml-cuda.h:30-32): give a
 * graph tensor device storage (scratch ring unless no_scratch). */
void   ggml_hip_assign_buffers(struct ggml_tensor *tensor);
void   ggml_hip_assign_buffers_no_scratch(struct ggml_tensor *tensor);
void   ggml_hip_assign_buffers_force_inplace(struct ggml_tensor *tensor);
/* ggml_cuda_set_main_device / set_scratch_size / free_scratch (ggml-cuda.h:33-35). */
void   ggml_hip_set_main_device(int main_device);
void   ggml_hip_set_scratch_size(size_t scratch_size);
void   ggml_hip_free_scratch(void);
/* ggml_cuda_compute_forward (ggml-cuda.h:36, ggml-cuda.cu:2933-3021): returns true when the
 * node was taken by the backend (the CPU op is then skipped, ggml.c:15645-15652).  Only thread
 * ith == 0 in the COMPUTE phase launches; the other threads/phases return true immediately. */
bool   ggml_hip_compute_forward(struct ggml_compute_params *params, struct ggml_tensor *tensor);
/* ggml_cpu_has_cublas (ggml.c:19465-19470) equivalent: 1 when a HIP device is usable. */
int    ggml_cpu_has_hipblas(void);

/* Device weight-residency cache.  A CPU-backend Q4_0 src0 (the arch/
 * frontends never call transform_tensor; the reference re-uploads it every call,
 * ggml-cuda.cu:2496-2502) is uploaded once per device and reused while a sampled fingerprint of
 * its bytes is unchanged; LRU under GGML_HIP_WEIGHT_CACHE_MB (default 65536), off with
 * GGML_HIP_WEIGHT_CACHE=0.  Counters since the last clear; clear frees every cached copy. */
int    ggml_hip_weight_cache_stats(int64_t *hits, int64_t *misses, int64_t *resident_bytes);
int    ggml_hip_weight_cache_clear(void);
/* Host writes into cached weights.  Writes made by ggml nodes (the reference's LoRA apply rewrites
 * Q4_0 weights in place through ggml_add_inplace / ggml_cpy graphs, llama.cpp:2950-2967) are seen
 * by ggml_hip_compute_forward's INIT phase and invalidate the overlapping copies exactly.  A host
 * that edits weight bytes outside ggml calls ggml_hip_weight_cache_invalidate(ptr, bytes) (drops
 * every copy overlapping [ptr, ptr+bytes), bytes 0 = the copies containing ptr; returns how many,
 * or a negative status), or runs with GGML_HIP_WEIGHT_CACHE_VERIFY=full / set_verify(1): every
 * lookup then fingerprints every byte of the host weight (exact; one host read per call; -1 =
 * environment, 0 = sampled fingerprint). */
int64_t ggml_hip_weight_cache_invalidate(const void *host, size_t bytes);
int    ggml_hip_weight_cache_set_verify(int mode);
int64_t ggml_hip_weight_cache_invalidations(void);

/* ------------------------------------------------------------------------------------------
 * Tensor-free entry points (device pointers, stream-ordered on `stream` = hipStream_t or NULL
 * for the backend's stream on the current device).  Return enum ggml_hip_status.
 * Layouts: ggml's.  W = block_q4_0 rows (18*K/32 bytes per row), x = f32 [N][K] row-major,
 * y = f32 [N][M] row-major (y[n*M + m], i.e. ggml dst with ne0 = M, ne1 = N).
 * Pointers must be 16-byte aligned; K % 64 == 0 (ggml.c:2344 asserts nb % 2 == 0).
 * ---------------------------------------------------------------------------------------- */

/* q8_0 quantize of N activation rows, ggml block_q8_0 output (34*K/32 bytes per row);
 * bit-exact to quantize_row_q8_0's AVX2 branch (ggml.c:1192-1275). */
int ggml_hip_quantize_q8_0(const float *dev_x, int64_t K, int64_t N, void *dev_xq, void *stream);
/* q4_0 weight quantizer, bit-exact to quantize_row_q4_0_reference (ggml.c:918-953). */
int ggml_hip_quantize_q4_0(const float *dev_w, int64_t K, int64_t M, void *dev_wq, void *stream);
/* dequantize_row_q4_0 (ggml.c:1500-1518). */
int ggml_hip_dequantize_q4_0(const void *dev_wq, int64_t K, int64_t M, float *dev_w, void *stream);

/* y = W x (ggml_compute_forward_mul_mat_q_f32, ggml.c:11226-11424, INIT + COMPUTE fused):
 * N <= 8: fused quantize + GEMV (one wave64 per weight row); N > 8: q8_0 quantize + int8-MFMA
 * GEMM.  Uses the backend's device workspace for N > 8 (grown outside stream capture by
 * ggml_hip_reserve_workspace or the first call). */
int ggml_hip_mul_mat_q4_0(const void *dev_w, int64_t K, int64_t M, const float *dev_x, int64_t N,
                          float *dev_y, void *stream);
/* Same with an explicit algorithm and output stride ldy: 0 auto (4 in exact mode; else 1 for N <= 8,
 * 3 for N <= 128, else 2), 1 fused GEMV (N <= 8), 2 LDS-staged int8-MFMA GEMM, 3 split-K int8-MFMA
 * GEMM (small N), 4 exact: every y bit-identical to the reference's x86 AVX2+FMA
 * ggml_vec_dot_q4_0_q8_0 (ggml.c:2412-2435; same q8_0 bytes, same fp32 fma schedule). */
int ggml_hip_mul_mat_q4_0_ex(const void *dev_w, int64_t K, int64_t M, const float *dev_x, int64_t N,
                             float *dev_y, int64_t ldy, int algo, void *stream);
/* Sibling mul_mats that share the activation x (ggml graphs issue wq/wk/wv and w1/w3 on the same
 * src1): n <= 4 weight matrices of the same K, y_i = W_i x with y_i f32 [N][M_i].  One launch for
 * N <= 8 (rows concatenated); for N > 8 x is quantized once and each W_i runs the GEMM.  Results
 * are identical to n separate ggml_hip_mul_mat_q4_0 calls, except where siblings with fp6 weight images
 * run as one prefill launch whose tile plan (128 x 64 / 128 x 128, by the launch's tile count) differs from
 * the single calls' (within the oracle bound; bitwise with ggml_hip_debug_set_gemm9_wide pinning the tile). */
int ggml_hip_mul_mat_q4_0_multi(int n, const void *const *dev_w, const int64_t *M, int64_t K, const float *dev_x,
                                int64_t N, float *const *dev_y, void *stream);
/* Exact (reproducible) mode, process-wide: every auto-selected mul_mat, including the ggml hook
 * path (ggml_hip_mul_mat / ggml_hip_compute_forward) and the sibling-matrix calls, runs algorithm 4,
 * so a ggml graph on this backend reproduces the reference CPU build's mul_mat outputs bit for bit.
 * Default off (GGML_HIP_EXACT=1 switches it on at first use); the fast kernels stay within the
 * north-star 1e-3 tolerance.  No ggml-cuda.h counterpart. */
int ggml_hip_set_exact(int on);
int ggml_hip_get_exact(void);
/* Ensure the current device's workspace can serve mul_mat for N tokens of K (call before
 * capturing a HIP graph). */
int ggml_hip_reserve_workspace(int64_t K, int64_t N);
/* The same for prefill mul_mats (N > 128) of matrices up to M rows: the LDS GEMM also keeps a per-call
 * image of the weights in the workspace (up to 34 bytes per 32 weights). */
int ggml_hip_reserve_workspace_mm(int64_t K, int64_t N, int64_t M);

/* Prefill weight images (no ggml-cuda.h counterpart).  The LDS GEMM (N > 64 with an image, N > 128 without) runs fastest on an image
 * of the weight: by default fp6 (e2m3 codes of w/2, w = nibble - 8, fp16 d verbatim; 26 B per 32
 * weights, 1.44x the q4_0 bytes; the exact block sums on the block-scaled fp6 MFMA, k_gemm9), under GEMM
 * version 8 int8 (34 B per 32 weights, k_gemm8; bitwise the same results): create builds it once
 * (stream-ordered, outside capture) and every later prefill mul_mat of that device pointer with the
 * same K, M uses it; without one the GEMM reads the q4_0 bytes directly.  The weight
 * must not change while its image exists (free it first).  Device-resident ggml weights
 * (transform_tensor, the residency cache) get their image on their first prefill use, dropped with the
 * buffer.  Results are identical either way in exact arithmetic per block; the fp32 accumulation order
 * of the two GEMMs differs (both within the parity bound). */
int ggml_hip_weight_image_create(const void *dev_w, int64_t K, int64_t M, void *stream);
int ggml_hip_weight_image_free(const void *dev_w);        /* number of images dropped */
int64_t ggml_hip_weight_image_bytes(void);                  /* device bytes held by images */
/* test hook: prefill GEMM version 7 (q4_0 bytes), 8 / 10 (int8 / fp6 images built on registration, the
 * GEMM of the image when one exists; 10 is the default), 9 / 11 (k_gemm8 / k_gemm9 always, an
 * unregistered weight converted per call into the workspace); -1 = GGML_HIP_GEMM_V */
int ggml_hip_debug_set_gemm_version(int v);
// k_gemm9's tile: -1 = automatic (128 x 128 where it takes fewer CU rounds than 128 x 64; GGML_HIP_GEMM9_WIDE
// overrides), 0 = always 128 x 64, 1 = always 128 x 128 (block order: y within the oracle bound of 128 x 64's).
int ggml_hip_debug_set_gemm9_wide(int mode);

/* ------------------------------------------------------------------------------------------
 * Decode chains: a sequence of dependent N = 1 q4_0 mul_mats, validated once and launched together.
 * A decode eval issues its q4_0 mul_mats one after another on one stream (llama.cpp:1217-1600 ->
 * ggml_compute_forward_mul_mat_q_f32, ggml.c:11226-11411).  A chain runs tasks 0..n-1 in stream order,
 * each as one sibling GEMV launch (ggml_hip_mul_mat_q4_0_multi with N = 1): task t reads x only after
 * every task < t has written its y, so x of a task may be, or overlap, the y of an earlier task.
 * Results are bitwise those of n separate ggml_hip_mul_mat_q4_0_multi calls (exact mode included).
 * A task's y must not overlap its own x (create rejects it).  Graph-capturable.  Two in-launch
 * designs (one persistent launch, round 2; overlapped launches with flag hand-offs, round 4) were
 * bitwise equal and slower.  No ggml-cuda.h counterpart.
 * ---------------------------------------------------------------------------------------- */
typedef struct ggml_hip_chain_task {
    int nmat;                 /* 1..4 sibling matrices sharing x (e.g. wq|wk|wv) */
    int64_t K;                /* K % 64 == 0 */
    const float *x;           /* f32 [K], 16-byte aligned */
    const void *W[4];         /* block_q4_0 rows, M[i] x K, 16-byte aligned */
    int64_t M[4];
    float *y[4];              /* f32 [M[i]] */
} ggml_hip_chain_task;
typedef struct ggml_hip_chain ggml_hip_chain;
/* Validates the tasks (no device work). */
int ggml_hip_chain_create(int ntasks, const ggml_hip_chain_task *tasks, ggml_hip_chain **chain);
/* N-token chains (prefill): x of a task is f32 [N][K], y[i] f32 [N][M[i]]; otherwise as above, bitwise n
 * separate ggml_hip_mul_mat_q4_0_multi calls at N.  A task whose siblings take one k_gemm9 launch on fp6
 * weight images (ggml_hip_weight_image_create) reads a chain-owned x image (gemm9 x bytes per task,
 * allocated at create), built by k_prep9_x; with the epilogue fold on (ggml_hip_debug_set_chain_x9(1)), a
 * task whose x is exactly y[i] of an earlier such task (M[i] == K, nothing in between writes it) gets it
 * from that task's GEMM epilogue instead (bitwise the same; measured slower, so off by default). */
int ggml_hip_chain_create_n(int ntasks, const ggml_hip_chain_task *tasks, int64_t N, ggml_hip_chain **chain);
/* debug: 1 = N-token chains take x images from the producers' GEMM epilogues, 0 = every image by
 * k_prep9_x (default), -1 = GGML_HIP_CHAIN_X9 (1 turns the fold on) */
int ggml_hip_debug_set_chain_x9(int on);
/* debug, no device needed: the epilogue links ggml_hip_chain_create_n would plan; prod[t] = the task whose
 * epilogue writes task t's x image (-1: k_prep9_x), share[t] = the earlier consumer whose image t reads (-1) */
int ggml_hip_debug_chain_links(int ntasks, const ggml_hip_chain_task *tasks, int64_t N, int *prod, int *share);
/* Stream-ordered (graph-capturable): one GEMV launch per task. */
int ggml_hip_chain_launch(ggml_hip_chain *chain, void *stream);
/* Synchronizes the device; 0, or (engine) the nonzero error bits of a bounded wait that expired. */
int ggml_hip_chain_status(ggml_hip_chain *chain);
int ggml_hip_chain_destroy(ggml_hip_chain *chain);
/* The persistent decode engine: the whole chain as ONE launch, one workgroup per CU, a loader
 * wave streaming each CU's weight rows by LDS-DMA ahead across the dependency edges, the edges carried by q8_0
 * blocks quantized once by their producer.  Results are bitwise those of the per-launch chain.  It takes chains
 * in which every task t >= 1 reads x = y[i] of task t - 1 (the same pointer, its first K values), task 0 reads an
 * x that no task writes, K <= 12288, and any output region written again later is ordered by the edges; other
 * chains, and every launch in exact mode, keep the per-launch path.  It needs the device to itself while it
 * runs (all workgroups co-resident); every wait is bounded (GGML_HIP_ENGINE_TIMEOUT_MS, default 2000) and
 * chain_status reports an expired one.  mode 1 on (builds the plan; returns 1 when the engine runs the chain, 0
 * when it declined: ggml_hip_last_error says why), 0 off, -1 query.  GGML_HIP_CHAIN_ENGINE=1 turns it on at
 * create.  info: [0] engine on, [1] work units, [2] largest per-CU stream (bytes), [3] weight bytes, [4] CUs,
 * [5] (N-token chains) tasks whose x image a producer's GEMM epilogue writes. */
int ggml_hip_chain_set_engine(ggml_hip_chain *chain, int mode);
int ggml_hip_chain_engine_info(ggml_hip_chain *chain, int64_t *info, int n);

/* ------------------------------------------------------------------------------------------
 * Multi-GPU, one process per GPU (torch.distributed-style ranks), RCCL over xGMI.
 * The reference row-splits weights across devices (GGML_BACKEND_GPU_SPLIT, ggml-cuda.cu:
 * 2361-2368, 2773-2806) and gathers each device's dst rows with cudaMemcpyAsync
 * (ggml-cuda.cu:2514-2539); here every rank holds rows [row_begin[rank], row_begin[rank+1])
 * and the slices are exchanged with one ncclAllGather.
 * ---------------------------------------------------------------------------------------- */
typedef struct ggml_hip_comm ggml_hip_comm;

#define GGML_HIP_UNIQUE_ID_BYTES 128
/* rank 0 creates the id and ships it to the other ranks (e.g. torch.distributed broadcast). */
int ggml_hip_comm_unique_id(char out[GGML_HIP_UNIQUE_ID_BYTES]);
int ggml_hip_comm_init(ggml_hip_comm **comm, int nranks, int rank, const char id[GGML_HIP_UNIQUE_ID_BYTES]);
int ggml_hip_comm_destroy(ggml_hip_comm *comm);
/* In-process loopback group (testing / single-process multi-device): creates nranks
 * communicators comms[0..nranks-1] whose all-gather has ncclAllGather's semantics, for nranks
 * host threads of this process that each drive one rank (rank r on devices[r], or all on the
 * current device when devices is NULL; give each rank its own stream).  Every split entry point
 * below runs the same code on either transport.  Destroy each comm with ggml_hip_comm_destroy. */
int ggml_hip_comm_init_local(ggml_hip_comm **comms, int nranks, const int *devices);
/* One process per rank without RCCL: the comm's host collectives (allreduce_host, the P2P handle
 * exchange) go through files in dir, a directory every rank can read and write (rank r writes
 * <dir>/c<nonce>_<seq>_r<r>).  Init is collective: rank 0 publishes a fresh session nonce as <dir>/session
 * and refuses a directory where that name exists (a session in progress or a crashed one's leftover), so
 * files of different sessions never mix.  Device all-gathers need the P2P transport (ggml_hip_comm_enable_p2p); the RCCL
 * transport is unavailable.  It also lets several processes share ONE device (RCCL refuses that),
 * which is how the cross-process IPC path of the P2P all-gather is tested on a one-GPU box. */
int ggml_hip_comm_init_file(ggml_hip_comm **comm, int nranks, int rank, const char *dir);
int ggml_hip_comm_rank(const ggml_hip_comm *comm, int *rank, int *nranks);
/* Direct-store all-gather (SURVEY.md §8e's P2P alternative to ncclAllGather for latency-bound decode
 * gathers): each rank stores its slice straight into every peer's landing buffer over xGMI (an IPC
 * mapping across processes, the buffer itself in a loopback group) and raises a flag there; one
 * kernel per all-gather, graph-capturable (the epoch advances on the device).  Collective: call on
 * every rank of the comm with the same max_floats (the largest slice of one all-gather, floats);
 * at most 8 ranks.  After it the comm's all-gathers (the split mul_mats) use P2P stores;
 * set_transport(comm, 0) returns to RCCL (1 = P2P again).  Every rank takes part in every collective of
 * enable_p2p and the outcome is the group's: all ranks enable it or all return an error.
 * Failure: a peer's data that does not arrive within the timeout (set_p2p_timeout, ms; <= 0 selects
 * GGML_HIP_P2P_TIMEOUT_MS, default 10000) FAILS the comm for good: that gather writes NaN into the
 * peer's segment (never the stale landing slot), later gathers fill every peer segment with NaN
 * without waiting, and the next split mul_mat / all-gather on the comm returns GGML_HIP_ERR_COMM
 * before enqueueing anything (the reference stops at its first failed copy, CUDA_CHECK,
 * ggml-cuda.cu:22-51).  The rank that sees a failure first notifies every peer (a failure word stored
 * into each peer's control block over the same mapping), and the peers' waits poll it, so every rank
 * fails within one poll instead of after its own timeout.  p2p_status synchronizes the device and
 * returns 0, or the bit mask of peers whose data never arrived or that reported a failure (sticky).
 * comm_abort fails this rank's comm on purpose and sends the same notice (ncclCommAbort's role; the
 * timeout is a kernel argument, so gathers captured in a HIP graph keep the value of their capture). */
int ggml_hip_comm_enable_p2p(ggml_hip_comm *comm, int64_t max_floats);
int ggml_hip_comm_set_transport(ggml_hip_comm *comm, int transport);
int ggml_hip_comm_p2p_status(ggml_hip_comm *comm);
int ggml_hip_comm_set_p2p_timeout(ggml_hip_comm *comm, double ms);
int ggml_hip_comm_abort(ggml_hip_comm *comm);
/* All-reduce of n <= 64 host doubles in place (op 0 sum, 1 max, 2 min) over the comm; synchronous,
 * so it is also a barrier (bench harness: max-over-ranks timing without a second runtime). */
int ggml_hip_comm_allreduce_host(ggml_hip_comm *comm, double *vals, int n, int op);
/* All-gather of host bytes: recv[r * bytes ...] = rank r's send (every transport; synchronous). */
int ggml_hip_comm_allgather_host(ggml_hip_comm *comm, const void *send, size_t bytes, void *recv);
/* Row split of M rows over nranks by cumulative fractions (NULL = equal split), the same
 * rule as the reference's tensor_split (ggml-cuda.cu:1863-1882, 2361-2368).  row_begin has
 * nranks+1 entries. */
int ggml_hip_split_rows(int64_t M, int nranks, const float *tensor_split, int64_t *row_begin);
/* y_full[N][M_total] = W_full x on every rank; this rank holds W rows
 * [row_begin[rank], row_begin[rank+1]) in dev_w_local (block_q4_0 rows).  Equal splits with
 * N == 1 gather straight into y_full; otherwise through a padded slab + compaction. */
int ggml_hip_mul_mat_q4_0_split(ggml_hip_comm *comm, const void *dev_w_local, int64_t K, int64_t M_total,
                                const int64_t *row_begin, const float *dev_x, int64_t N, float *dev_y_full,
                                void *stream);
/* Sibling form ("fuse QKV (3) and w1/w3 (2) into one all-gather each"): n <= 4
 * matrices sharing x, matrix i row-split by row_begin[i] (nranks+1 entries each).  With equal
 * splits and N == 1 this rank's slices are computed by ONE multi-matrix GEMV launch straight into
 * their places in y_full[i], then ONE grouped RCCL all-gather (ncclGroupStart/End) completes all
 * n outputs in place.  Other cases run ggml_hip_mul_mat_q4_0_split per matrix.  Results are
 * identical to n separate split calls. */
int ggml_hip_mul_mat_q4_0_split_multi(ggml_hip_comm *comm, int n, const void *const *dev_w_local, const int64_t *M_total,
                                      const int64_t *const *row_begin, int64_t K, const float *dev_x, int64_t N,
                                      float *const *dev_y_full, void *stream);

/* ------------------------------------------------------------------------------------------
 * Device plumbing for bindings (ctypes / cgo / JNI) that have no HIP headers.
 * ---------------------------------------------------------------------------------------- */
int    ggml_hip_device_count(void);
int    ggml_hip_set_device(int device);
int    ggml_hip_get_device(void);
void  *ggml_hip_dev_malloc(size_t size);
void   ggml_hip_dev_free(void *ptr);
int    ggml_hip_memcpy_h2d(void *dst, const void *src, size_t size, void *stream);
int    ggml_hip_memcpy_d2h(void *dst, const void *src, size_t size, void *stream);
int    ggml_hip_memcpy_d2d(void *dst, const void *src, size_t size, void *stream);
int    ggml_hip_memset(void *dst, int value, size_t size, void *stream);
int    ggml_hip_stream_synchronize(void *stream);
int    ggml_hip_device_synchronize(void);
void  *ggml_hip_default_stream(void);          /* the backend's stream on the current device */
void  *ggml_hip_stream_create(void);           /* a non-blocking stream on the current device */
int    ggml_hip_stream_destroy(void *stream);  /* synchronizes, frees its mul_mat workspace */
int    ggml_hip_fill_gaussian(float *dev_dst, int64_t n, uint64_t seed, float mean, float stdv, void *stream);
/* timing and HIP-graph capture on a stream (bench harness; launch-bound decode chains) */
void  *ggml_hip_event_create(void);
int    ggml_hip_event_record(void *event, void *stream);
float  ggml_hip_event_elapsed_ms(void *start, void *stop);   /* waits for stop */
void   ggml_hip_event_destroy(void *event);
typedef struct ggml_hip_graph ggml_hip_graph;
int    ggml_hip_graph_begin(void *stream);
int    ggml_hip_graph_end(void *stream, ggml_hip_graph **graph);
int    ggml_hip_graph_launch(ggml_hip_graph *graph, void *stream);
int    ggml_hip_graph_destroy(ggml_hip_graph *graph);
const char *ggml_hip_last_error(void);
const char *ggml_hip_version(void);
/* debug: counts[op] = device nodes run per ggml op (GGML_OP_COUNT = 68 slots), counts[68] = host ns
   inside ggml_hip_compute_forward, counts[69 + op] = that host time per op of the arriving node,
   counts[137 + k] = fused launches of chain k (0 add/rms_norm/mul, 1 scale/diag_mask_inf/soft_max,
   2 silu/mul, 3 rope/cpy, 4 f16 mul_mat/permute/cpy, 5 q4_0 mul_mat run while a silu is pending,
   6 sibling q4_0 GEMVs sharing src1 run as one group: wq|wk|wv, w1|w3, 7 independent rope /
   rope->cpy / cpy nodes held behind a group run as one launch, 8 decode scale -> diag_mask_inf ->
   soft_max -> KQV -> merged copy as one launch, 9 / 10 decode norm / silu chain run in the q4_0
   GEMV prologue, 11 prefill norm / silu chain that wrote the k_gemm9 x image of its output for the
   q4_0 mul_mats consuming it) */
int    ggml_hip_debug_op_stats(int64_t *counts, int n, int reset);
/* debug: the attention's f16 x f32 mul_mat on device pointers (synchronous); tiled = 0 one 32-lane
   group per output, 1 the LDS-tiled kernel, -1 the backend's choice (bit-identical either way) */
int    ggml_hip_debug_f16_mul_mat(const void *s0, const void *s1, float *d, int K, int64_t ne01, int64_t ne11,
                                  int64_t ne02, int64_t nb01, int64_t nb02, int64_t nb11, int64_t nb12,
                                  float *merged, int tiled);
/* debug: mode-0 rope (ggml_compute_forward_rope_f32) of x [ne2 tokens][ne1 heads][ne0] (byte strides
   nbx[1..3]) into d (nbd[1..3]) at positions n_past.., then (c != nullptr) ggml_cpy of d into the view c
   (F16 when to_f16; shape ne10 x ne11 x .., byte strides nb10..nb12); batched = 1 through the batched
   elementwise launch (as the hook runs rope K -> K cache behind a q4_0 group), 0 its own kernel */
int    ggml_hip_debug_rope(const void *x, void *d, void *c, int to_f16, int64_t ne0, int64_t ne1, int64_t ne2,
                           int n_past, int n_dims, const int64_t *nbx, const int64_t *nbd, int64_t ne10,
                           int64_t ne11, int64_t nb10, int64_t nb11, int64_t nb12, int batched);
/* debug: ggml_cpy F32 -> F32 / F16 (to_f16) on device pointers (synchronous): source shape ne00 x ne01 x
   n / (ne00 ne01) with byte strides nb00..nb02, target ne10 x ne11 x .. with nb10..nb12; batched = 1
   through the batched elementwise launch (as the hook runs it behind a q4_0 group), 0 as its own node */
int    ggml_hip_debug_cpy_f32(const void *x, void *d, int to_f16, int64_t n, int64_t ne00, int64_t ne01,
                              int64_t nb00, int64_t nb01, int64_t nb02, int64_t ne10, int64_t ne11, int64_t nb10,
                              int64_t nb11, int64_t nb12, int batched);
/* debug: 1/0 = launch fusion of adjacent full-offload nodes on/off (default: env GGML_HIP_FUSE, on) */
int    ggml_hip_debug_set_fuse(int on);

#ifdef __cplusplus
}
#endif

#endif /* GGML_HIP_H */
