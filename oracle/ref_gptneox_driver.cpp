// ref_gptneox_driver.cpp — TEST INFRASTRUCTURE ONLY (the caller side, like ref_falcon_driver.cpp): the
// reference's own GPT-NeoX frontend (arch/gptneox/gptneox.cpp: its GGJT v1 loader, gptneox.cpp:420-540,
// and its eval graph, gptneox_eval_internal 1085-) compiled from /root/reference with the reference's
// ggml.c.  Built twice by oracle/Makefile: CPU-only (the golden side) and with -DGGML_USE_CUBLAS linked
// against libggml_hip_cuda.so.  Like every arch/ frontend it never offloads a tensor, so in the second
// build ggml.c's hooks send each Q4_0 mul_mat the backend's can_mul_mat accepts to the MI355X (weights
// from the device residency cache); everything else runs on ggml's CPU ops.
#include "arch/gptneox/gptneox.h"

#include <cstring>

// Evaluates the prompt (tokens[0..n_tokens) at n_past = 0), then n_decode single-token steps
// (decode_tokens[i] at n_past = n_tokens + i).  prompt_out receives the last prompt row of logits,
// decode_out[i * n_vocab ...] the logits of decode step i.  Returns n_vocab, or < 0 on error.
extern "C" int refgptneox_logits(const char *path, const int *tokens, int n_tokens, const int *decode_tokens,
                                 int n_decode, int n_threads, float *prompt_out, float *decode_out) {
    gptneox_context_params p = gptneox_context_default_params();
    p.n_ctx = 128;
    p.seed = 1;
    p.use_mmap = false;
    gptneox_context *c = gptneox_init_from_file(path, p);
    if (!c) return -1;
    const int nv = gptneox_n_vocab(c);
    int rc = gptneox_eval(c, (const gptneox_token *)tokens, n_tokens, 0, n_threads) ? -2 : 0;
    if (rc == 0) memcpy(prompt_out, gptneox_get_logits(c), sizeof(float) * (size_t)nv);
    for (int i = 0; i < n_decode && rc == 0; i++) {
        rc = gptneox_eval(c, (const gptneox_token *)&decode_tokens[i], 1, n_tokens + i, n_threads) ? -3 : 0;
        if (rc == 0) memcpy(decode_out + (size_t)i * nv, gptneox_get_logits(c), sizeof(float) * (size_t)nv);
    }
    gptneox_free(c);
    return rc == 0 ? nv : rc;
}
