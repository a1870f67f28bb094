// ggml-hip-internal.h — declarations shared by the host translation units of libggml_hip.so (not installed;
// the public C ABI is include/ggml-hip.h).  One seam per file:
//   ggml-hip-core.cpp    per-device state, temporaries, workspaces, the device-pointer mul_mat core
//   ggml-hip-wcache.cpp  prefill weight images and the residency cache of CPU-backend weights
//   ggml-hip-api.cpp     the tensor-free C ABI and device plumbing
//   ggml-hip-tensor.cpp  the ggml tensor ABI (ggml-cuda.h restated), ggml_hip_compute_forward
//   ggml-hip-fuse.cpp    the hook's node scheduler: held nodes, launch fusion, sibling groups
//   ggml-hip-ops.cpp     the non-Q4_0 device ops of a LLaMA layer
//   ggml-hip-comm.cpp    communicators, the P2P all-gather, row-split mul_mats
#pragma once

#include "../../include/ggml-hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ggml_abi.h"
#include "ggml_ops.h"
#include "launch.h"
#include "q4_0_kernels.h"

// Every HIP / RCCL call of the backend that is not a kernel launch first submits the launches the
// recorder holds (launch.h), so stream order is the order the backend issued its work in.
#define GHIP_SYNC(f) (ghip::rec_flush_at(#f " @" GHIP_STR(__LINE__)), f)
#define GHIP_STR2(x) #x
#define GHIP_STR(x) GHIP_STR2(x)

// errors: the tensor ABI is fail-fast like CUDA_CHECK (ggml-cuda.cu:22-51); the tensor-free ABI returns a
// status and keeps the message for ggml_hip_last_error()
#define HIP_FATAL(expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "ggml-hip: HIP error %d at %s:%d: %s\n", (int)e_, __FILE__, __LINE__,     \
                    hipGetErrorString(e_));                                                          \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

#define HIP_RET(expr)                                                                                \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            ::ghh::g_last_error = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return GGML_HIP_ERR_DEVICE;                                                              \
        }                                                                                            \
    } while (0)

// ---- the persistent decode engine (q4_0_engine.hip): a chain of dependent N = 1 mul_mats as one launch
namespace ghip {
struct EnginePlan;
EnginePlan *engine_plan_create(int ntasks, const ggml_hip_chain_task *tasks, int ncu, uint32_t timeout_ticks,
                               std::string &why);
hipError_t engine_launch(EnginePlan *p, hipStream_t s);
int engine_status(EnginePlan *p, uint64_t *detail);
void engine_plan_destroy(EnginePlan *p);
void engine_plan_info(const EnginePlan *p, int64_t *info);   // units, max CU stream bytes, weight bytes, CUs
int engine_stamps(EnginePlan *p, uint64_t *out, int64_t n);
}  // namespace ghip

namespace ghh {

using gabi::tensor;

constexpr int QK = 32;
constexpr int Q4B = 18;

extern thread_local std::string g_last_error;
int fail(int code, const std::string &msg);

// ---- per-device state (ggml-hip-core.cpp)
struct PoolBuf {
    void *ptr;
    size_t size;
};

struct Device {
    hipStream_t stream = nullptr;
    ghip::DeviceInfo info{};
    size_t total_mem = 0;
    std::mutex mu;
    std::vector<PoolBuf> pool;           // free temporaries (first-fit best size)
    void *ws = nullptr;                  // mul_mat workspace (q8_0 activations) of `stream`
    size_t ws_size = 0;
    // workspaces of other streams on this device (callers that run mul_mats on their own streams
    // concurrently, e.g. the ranks of an in-process loopback group): one per stream, never shared
    std::unordered_map<hipStream_t, PoolBuf> stream_ws;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;   // split mul_mat ordering between device streams
};

extern int g_device_count;
extern Device *g_dev;
extern int g_main_device;
extern float g_tensor_split[GGML_HIP_MAX_DEVICES];
extern size_t g_scratch_size;
extern void *g_scratch;
extern size_t g_scratch_offset;
extern bool g_eval_computed;            // a node ran since the last buffer assignment

// ggml-cuda.cu:1874-1881: cumulative start fractions in float, each divided by the float sum
inline void split_fractions(const float *tensor_split, int n, float *frac) {
    float split_sum = 0.0f;
    for (int i = 0; i < n; i++) {
        frac[i] = split_sum;
        split_sum += tensor_split[i];
    }
    for (int i = 0; i < n; i++) frac[i] /= split_sum;
}

// ggml-cuda.cu:2363, 2785: row_low = nrows0*g_tensor_split[id] -- int64*float is a float product
inline int64_t split_row_low(int64_t nrows, const float *frac, int id) {
    return id == 0 ? 0 : (int64_t)(nrows * frac[id]);
}

void ensure_init();
int current_device();
hipStream_t resolve_stream(void *stream);
void *pool_malloc(int id, size_t size, size_t *actual);
void pool_free(int id, void *p, size_t size);
size_t ws_d16_offset(int64_t K, int64_t N);
size_t workspace_bytes(int64_t K, int64_t N);
size_t ws_g8x_offset(int64_t K, int64_t N);
size_t ws_g8w_offset(int64_t K, int64_t N);
size_t workspace_bytes_mm(int64_t K, int64_t N, int64_t M);
extern std::atomic<int> g_gemm_v;
int gemm_version();
int reserve_workspace(int id, size_t bytes, hipStream_t s = nullptr);
int stream_workspace(int id, hipStream_t s, size_t need, void **out);
bool aligned(const void *p, size_t a);

// ---- the mul_mat core (ggml-hip-core.cpp)
extern std::atomic<int> g_exact;
bool exact_mode();
// xq: in/out mask of the q8_0(x) forms already in this stream's workspace from the previous call
enum { XQ_SOA = 1, XQ_G8 = 2, XQ_G9 = 4 };
int mul_mat_dev(const void *w, int64_t K, int64_t M, const float *x, int64_t N, float *y, int64_t ldy, int algo,
                hipStream_t s, unsigned *xq = nullptr);
int mul_mat_group_g9(int n, const void *const *w, const int64_t *M, int64_t K, const float *x, int64_t N,
                     float *const *y, hipStream_t s);
// true when ggml_hip_mul_mat_q4_0_multi runs these n siblings at N tokens as ONE k_gemm9 launch on registered
// fp6 images (mul_mat_group_g9 for n > 1, mul_mat_dev's image GEMM for n = 1); img[i] = the images
bool g9_images(int n, const void *const *w, const int64_t *M, int64_t K, int64_t N, const void **img);

// tensor helpers
bool is_contiguous(const tensor *t);
bool on_device(const tensor *t);
void split_range(int64_t nrows, int id, int64_t *lo, int64_t *hi);
bool supported_mul_mat(const tensor *src0, const tensor *src1, const tensor *dst);
[[noreturn]] void op_abort(const tensor *t, const char *why);
inline bool same_shape(const tensor *a, const tensor *b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}

// ---- weight images and the residency cache (ggml-hip-wcache.cpp)
int image_format();
// a weight with an image takes the image GEMM above this token count (below it the split-K GEMM on
// the q4_0 bytes; tools/n_sweep9.py: at N = 96 k_gemm9 24 / 26 / 51 us vs split-K 31 / 67 / 62 us for
// 4096^2 / 4096->11008 / 11008->4096, at N = 64 split-K still wins two of the three)
constexpr int64_t IMG_MIN_N = 64;
// ... and at any N above the GEMV's for tall matrices (4096 -> 11008: k_gemm9 23.4-24.6 us at N = 16-64
// against split-K 27.0-43.8, whose K walk streams every row per token tile)
constexpr int64_t IMG_MIN_M = 8192;
const void *wimage_find(int id, const void *w, int64_t K, int64_t M, int *fmt = nullptr);
const void *wimage_ensure(int id, const void *w, int64_t K, int64_t M, hipStream_t s);
int64_t wimage_drop(const void *dev, size_t bytes);
bool wcache_enabled();
int64_t decode_min_weights();
uint64_t wcache_next_call_id();
const void *wcache_get(int id, const void *host, size_t bytes, hipStream_t s, uint64_t call_id);
bool wcache_images_enabled();
void wcache_note_image(int id, const void *dev, size_t img_bytes, uint64_t call_id);
void wcache_image_dropped(const void *dev);
int64_t wcache_invalidate(const void *host, size_t bytes);
void wcache_note_host_write(const void *data, size_t bytes);

// ---- device ops (ggml-hip-ops.cpp)
struct OpTables {
    uint16_t *silu = nullptr;                // table_silu_f16 (ggml.c:4252), as the kernels get it (lut_apply)
    uint16_t *exp = nullptr;                 // table_exp_f16  (ggml.c:4253), the same
    uint16_t *silu_raw = nullptr, *exp_raw = nullptr;   // the device tables
    int silu_bad = -1, exp_bad = -1;         // finite inputs where the direct evaluation differs (device check)
};
const OpTables &op_tables(int id, hipStream_t s);
const float *rope_table(int id, int64_t ne0, int n_dims, int64_t need_pos, hipStream_t s);
void run_device_op(tensor *t, const tensor *fused_cpy = nullptr);
extern std::atomic<int64_t> g_op_count[gabi::OP_COUNT];      // device nodes run, per ggml op (debug stats)
extern std::atomic<int64_t> g_host_ns;                        // host time inside the taken nodes
extern std::atomic<int64_t> g_op_ns[gabi::OP_COUNT];          // the same, per op of the node that arrived
// fused launches by chain (index list at the definition, ggml-hip-ops.cpp)
constexpr int N_FUSED = 15;
extern std::atomic<int64_t> g_fused[N_FUSED];

// ---- the hook's node scheduler (ggml-hip-fuse.cpp)
void flush_deferred();                  // every backend entry point that can touch device memory
void execute_node(tensor *t);           // runs (or defers) one taken node
bool hook_holding();                    // any node held (pending chain, norm chain, group)
bool hook_seen(const tensor *t);        // t was snapshotted while held (a new graph at old addresses)
void snap_reset();
size_t span_bytes(const tensor *t);
bool graph_enabled();
int graph_apply_mode();

// ---- the tensor ABI (ggml-hip-tensor.cpp)
void mul_mat_node(const tensor *src0, const tensor *src1, tensor *dst);

}  // namespace ghh
