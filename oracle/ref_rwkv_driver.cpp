// ref_rwkv_driver.cpp — TEST INFRASTRUCTURE ONLY (the caller side, like ref_falcon_driver.cpp): the
// reference's own RWKV frontend (arch/rwkv/rwkv.cpp: its GGJT v1 loader, rwkv.cpp:500-610, and its
// recurrent one-token graph, rwkv_build_graph / rwkv_eval_internal 1683-) compiled from /root/reference
// with the reference's ggml.c.  Built twice by oracle/Makefile: CPU-only (the golden side) and with
// -DGGML_USE_CUBLAS linked against libggml_hip_cuda.so.  RWKV evaluates one token per graph (every Q4_0
// mul_mat is a decode GEMV, N = 1); the frontend never offloads a tensor, so in the second build
// ggml.c's hooks send each Q4_0 mul_mat the backend's can_mul_mat accepts to the MI355X (weights from
// the device residency cache); everything else, including the frontend's ggml_map_* custom ops,
// runs on ggml's CPU ops.
#include "arch/rwkv/rwkv.h"

#include <cstring>

// Evaluates tokens[0..n_tokens) one at a time (the recurrent state carries the prompt), then n_decode
// more tokens.  prompt_out receives the logits after the last prompt token, decode_out[i * n_vocab ...]
// those after decode token i.  Returns n_vocab, or < 0 on error.
extern "C" int refrwkv_logits(const char *path, const int *tokens, int n_tokens, const int *decode_tokens,
                              int n_decode, float *prompt_out, float *decode_out) {
    rwkv_context_params p = rwkv_context_default_params();
    p.seed = 1;
    p.use_mmap = false;
    rwkv_context *c = rwkv_init_from_file(path, p);
    if (!c) return -1;
    const int nv = rwkv_n_vocab(c);
    int rc = 0;
    for (int i = 0; i < n_tokens && rc == 0; i++) rc = rwkv_eval(c, (rwkv_token)tokens[i], nullptr) ? -2 : 0;
    if (rc == 0) memcpy(prompt_out, rwkv_get_logits(c), sizeof(float) * (size_t)nv);
    for (int i = 0; i < n_decode && rc == 0; i++) {
        rc = rwkv_eval(c, (rwkv_token)decode_tokens[i], nullptr) ? -3 : 0;
        if (rc == 0) memcpy(decode_out + (size_t)i * nv, rwkv_get_logits(c), sizeof(float) * (size_t)nv);
    }
    rwkv_free(c);
    return rc == 0 ? nv : rc;
}
