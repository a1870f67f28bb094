// Writes tests/golden/ggml_op_enum.json: the reference ggml.h enum values the backend mirrors
// (csrc/ggml_abi.h).  gcc -I/root/reference tests/golden/gen_ggml_enum.c -o /tmp/e && /tmp/e > tests/golden/ggml_op_enum.json
#include "ggml.h"
#include <stdio.h>
#include <stddef.h>
int main(void) {
    printf("{\"GGML_OP_ADD\": %d, \"GGML_OP_MUL\": %d, \"GGML_OP_SILU\": %d, \"GGML_OP_RMS_NORM\": %d, \"GGML_OP_MUL_MAT\": %d, "
           "\"GGML_OP_SCALE\": %d, \"GGML_OP_CPY\": %d, \"GGML_OP_RESHAPE\": %d, \"GGML_OP_VIEW\": %d, \"GGML_OP_PERMUTE\": %d, "
           "\"GGML_OP_TRANSPOSE\": %d, \"GGML_OP_DIAG_MASK_INF\": %d, \"GGML_OP_SOFT_MAX\": %d, \"GGML_OP_ROPE\": %d, "
           "\"GGML_OP_COUNT\": %d, \"GGML_TYPE_I32\": %d, \"GGML_TYPE_F16\": %d}\n",
           GGML_OP_ADD, GGML_OP_MUL, GGML_OP_SILU, GGML_OP_RMS_NORM, GGML_OP_MUL_MAT, GGML_OP_SCALE, GGML_OP_CPY,
           GGML_OP_RESHAPE, GGML_OP_VIEW, GGML_OP_PERMUTE, GGML_OP_TRANSPOSE, GGML_OP_DIAG_MASK_INF, GGML_OP_SOFT_MAX,
           GGML_OP_ROPE, GGML_OP_COUNT, GGML_TYPE_I32, GGML_TYPE_F16);
    return 0;
}
