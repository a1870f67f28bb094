// ggml_abi.h — bit-for-bit mirror of the reference ggml structs this backend reads.
//
// The backend links into an unmodified ggml.c, so it must agree with
// ggml.h:378-414 (struct ggml_tensor) and ggml.h:459-468 (struct ggml_compute_params) of
// Fcucgvhhhvjv/llama.cpp-q_4_0 — including the fork's four GGML_OP_EXT_* ops
// (ggml.h:314-317) that shift GGML_OP_MUL_MAT to 32.  The static_asserts pin the layout
// measured from the reference header.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace gabi {

constexpr int MAX_DIMS = 4;   // GGML_MAX_DIMS  ggml.h:196
constexpr int MAX_OPT = 4;    // GGML_MAX_OPT   ggml.h:200
constexpr int MAX_NAME = 48;  // GGML_MAX_NAME  ggml.h:201

enum type : int { TYPE_F32 = 0, TYPE_F16 = 1, TYPE_Q4_0 = 2, TYPE_Q8_0 = 8, TYPE_I32 = 18, TYPE_COUNT = 19 };
enum backend : int { BACKEND_CPU = 0, BACKEND_GPU = 10, BACKEND_GPU_SPLIT = 20 };   // ggml.h:257-261
// enum ggml_op (ggml.h:274-350, with the fork's GGML_OP_EXT_* at 28-31; tests/golden/ggml_op_enum.json)
enum op : int { OP_NONE = 0, OP_ADD = 2, OP_MUL = 6, OP_SILU = 23, OP_RMS_NORM = 26, OP_MUL_MAT = 32, OP_SCALE = 34,
                OP_CPY = 36, OP_RESHAPE = 38, OP_VIEW = 39, OP_PERMUTE = 40, OP_TRANSPOSE = 41,
                OP_DIAG_MASK_INF = 45, OP_SOFT_MAX = 47, OP_ROPE = 49, OP_COUNT = 68 };
enum task_type : int { TASK_INIT = 0, TASK_COMPUTE = 1, TASK_FINALIZE = 2 };

struct tensor {
    int type;
    int backend;
    int n_dims;
    int64_t ne[MAX_DIMS];
    size_t nb[MAX_DIMS];
    int op;
    bool is_param;
    tensor *grad;
    tensor *src0;
    tensor *src1;
    tensor *opt[MAX_OPT];
    int n_tasks;
    int perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;
    void *data;
    char name[MAX_NAME];
    void *extra;
    char padding[4];
};

struct compute_params {
    int type;       // enum ggml_task_type
    int ith, nth;
    size_t wsize;
    void *wdata;
};

static_assert(sizeof(tensor) == 240, "ggml_tensor size");
static_assert(offsetof(tensor, backend) == 4, "backend");
static_assert(offsetof(tensor, n_dims) == 8, "n_dims");
static_assert(offsetof(tensor, ne) == 16, "ne");
static_assert(offsetof(tensor, nb) == 48, "nb");
static_assert(offsetof(tensor, op) == 80, "op");
static_assert(offsetof(tensor, src0) == 96, "src0");
static_assert(offsetof(tensor, src1) == 104, "src1");
static_assert(offsetof(tensor, n_tasks) == 144, "n_tasks");
static_assert(offsetof(tensor, data) == 168, "data");
static_assert(offsetof(tensor, name) == 176, "name");
static_assert(offsetof(tensor, extra) == 224, "extra");
static_assert(sizeof(compute_params) == 32, "ggml_compute_params size");
static_assert(offsetof(compute_params, wsize) == 16, "wsize");
static_assert(offsetof(compute_params, wdata) == 24, "wdata");

// GGML_TYPE_SIZE / GGML_BLCK_SIZE for the types this backend touches (ggml.c:3586-3620)
inline size_t type_size(int t) {
    return t == TYPE_F32 || t == TYPE_I32 ? 4 : t == TYPE_F16 ? 2 : t == TYPE_Q4_0 ? 18 : t == TYPE_Q8_0 ? 34 : 0;
}
inline int blck_size(int t) { return (t == TYPE_Q4_0 || t == TYPE_Q8_0) ? 32 : 1; }
inline size_t nbytes(const tensor *t) {
    return (size_t)(t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]) * type_size(t->type) / blck_size(t->type);
}
inline int64_t nrows(const tensor *t) { return t->ne[1] * t->ne[2] * t->ne[3]; }

}  // namespace gabi
