// ref_falcon_driver.cpp — TEST INFRASTRUCTURE ONLY (the caller side, like ref_llama_driver.cpp): the
// reference's own Falcon frontend (arch/falcon/falcon.cpp: its GGJT v1 loader, falcon.cpp:417-535,
// and its eval graph, falcon_eval_internal 1124-1404) compiled from /root/reference with the
// reference's ggml.c.  Built twice by oracle/Makefile: CPU-only (the golden side) and with
// -DGGML_USE_CUBLAS linked against libggml_hip_cuda.so.  The arch frontends never offload a tensor
// (no transform_tensor, no assign_buffers: every weight is a CPU tensor), so in the second build
// ggml.c's hooks send each Q4_0 mul_mat the backend's can_mul_mat accepts to the MI355X, the weight
// served from the device residency cache; everything else runs on ggml's CPU ops.
#include "arch/falcon/falcon.h"

#include <cstdio>
#include <cstring>
#include <vector>

// Evaluates the prompt (tokens[0..n_tokens) at n_past = 0), then n_decode single-token steps
// (decode_tokens[i] at n_past = n_tokens + i).  prompt_out receives the last prompt row of logits,
// decode_out[i * n_vocab ...] the logits of decode step i.  Returns n_vocab, or < 0 on error.
extern "C" int reffalcon_logits(const char *path, const int *tokens, int n_tokens, const int *decode_tokens,
                                int n_decode, int n_threads, float *prompt_out, float *decode_out) {
    falcon_context_params p = falcon_context_default_params();
    p.n_ctx = 128;
    p.seed = 1;
    p.use_mmap = false;
    falcon_context *c = falcon_init_from_file(path, p);
    if (!c) return -1;
    const int nv = falcon_n_vocab(c);
    int rc = falcon_eval(c, (const falcon_token *)tokens, n_tokens, 0, n_threads) ? -2 : 0;
    if (rc == 0) memcpy(prompt_out, falcon_get_logits(c), sizeof(float) * (size_t)nv);
    for (int i = 0; i < n_decode && rc == 0; i++) {
        rc = falcon_eval(c, (const falcon_token *)&decode_tokens[i], 1, n_tokens + i, n_threads) ? -3 : 0;
        if (rc == 0) memcpy(decode_out + (size_t)i * nv, falcon_get_logits(c), sizeof(float) * (size_t)nv);
    }
    falcon_free(c);
    return rc == 0 ? nv : rc;
}
