// ref_llama_driver.cpp — TEST INFRASTRUCTURE ONLY (the caller side, like ref_hip_driver.c): the
// reference's own llama.cpp (its GGJT v3 loader, llama.cpp:383-503, and its eval graph) compiled
// from /root/reference, loads a model file and evaluates a prompt.  Built twice by oracle/Makefile:
// CPU-only (golden logits) and with -DGGML_USE_CUBLAS linked against libggml_hip_cuda.so, where
// ggml.c's hooks send every Q4_0 mul_mat of a >= 32-token batch to the MI355X backend (weights stay
// CPU tensors at n_gpu_layers = 0, the arch/-frontend situation, and hit the weight-residency cache;
// n_gpu_layers > 0 sends the offloaded layers' weights through the loader's transform_tensor).
#include "llama.h"

#include <execinfo.h>
#include <chrono>
#include <vector>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

static bool g_trace = false;
#define STAGE(msg) do { if (g_trace) { fprintf(stderr, "refllama: %s\n", msg); fflush(stderr); } } while (0)

static void refllama_segv(int sig) {   // REFLLAMA_BACKTRACE=1: native stack of a crash (no gdb here)
    void *f[64];
    const int n = backtrace(f, 64);
    backtrace_symbols_fd(f, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

// Evaluates the prompt (n_evals times from n_past = 0: repeated evals give the same logits), then
// n_decode single-token steps (tokens decode_tokens[i] at n_past = n_tokens + i), whose logits go
// to decode_out[i * n_vocab].  Returns n_vocab, or < 0 on error.
extern "C" int refllama_logits(const char *path, const int *tokens, int n_tokens, int n_threads, int logits_all,
                               float *out, int out_cap, int n_evals, int n_gpu_layers, const int *decode_tokens,
                               int n_decode, float *decode_out) {
    g_trace = getenv("REFLLAMA_BACKTRACE") != nullptr;
    if (g_trace) {   // own stack for the handler: a stack overflow must still print
        static char alt[1 << 16];
        stack_t ss{};
        ss.ss_sp = alt;
        ss.ss_size = sizeof(alt);
        sigaltstack(&ss, nullptr);
        struct sigaction sa {};
        sa.sa_handler = refllama_segv;
        sa.sa_flags = SA_ONSTACK;
        sigaction(SIGSEGV, &sa, nullptr);
    }
    llama_init_backend(false);
    STAGE("backend initialised");
    llama_context_params p = llama_context_default_params();
    p.n_ctx = 256;
    p.n_batch = 512;
    p.n_gpu_layers = n_gpu_layers;   // > 0: the loader uploads those layers (llama.cpp:678-685)
    p.seed = 1;
    p.use_mmap = getenv("REFLLAMA_NO_MMAP") == nullptr;
    p.logits_all = logits_all != 0;
    llama_model *m = llama_load_model_from_file(path, p);
    if (!m) return -1;
    STAGE("model loaded");
    llama_context *c = llama_new_context_with_model(m, p);
    if (!c) {
        llama_free_model(m);
        return -2;
    }
    STAGE("context created");
    int rc = 0;
    for (int e = 0; e < (n_evals > 0 ? n_evals : 1) && rc == 0; e++)   // repeated evals: same logits
        rc = llama_eval(c, (const llama_token *)tokens, n_tokens, 0, n_threads) ? -3 : 0;
    STAGE("evaluated");
    const int nv = llama_n_vocab(c);
    if (rc == 0) {
        const int rows = logits_all ? n_tokens : 1;
        const int cnt = rows * nv < out_cap ? rows * nv : out_cap;
        memcpy(out, llama_get_logits(c), sizeof(float) * (size_t)cnt);
        for (int i = 0; i < n_decode && rc == 0; i++) {
            rc = llama_eval(c, (const llama_token *)&decode_tokens[i], 1, n_tokens + i, n_threads) ? -4 : 0;
            if (rc == 0) memcpy(decode_out + (size_t)i * nv, llama_get_logits(c), sizeof(float) * (size_t)nv);
        }
        if (rc == 0) rc = nv;
    }
    llama_free(c);
    STAGE("context freed");
    llama_free_model(m);
    return rc;
}

// End-to-end timing (tools/e2e_llama.py): load, evaluate an n_prompt-token prompt (reps times from
// n_past = 0), then n_decode single-token evals; wall times via steady_clock around llama_eval.
// out[0] = load s, out[1] = prompt ms (mean over reps), out[2] = decode ms per token; the logits of
// the last decode step go to last_logits[0..n_vocab).  Returns n_vocab or < 0.
// min / max over the reps of the last refllama_bench call's prompt evals (the first rep also builds the
// backend's weight images; the min is the steady state)
static double g_prompt_min_ms = 0.0, g_prompt_max_ms = 0.0;
extern "C" void refllama_last_prompt_range(double *min_ms, double *max_ms) {
    *min_ms = g_prompt_min_ms;
    *max_ms = g_prompt_max_ms;
}

extern "C" int refllama_bench(const char *path, int n_prompt, int n_decode, int n_threads, int n_gpu_layers, int n_ctx,
                              int reps, double *out, float *last_logits) {
    using clk = std::chrono::steady_clock;
    // llama_eval does not check n_past + N <= n_ctx; past it the KV-cache views run off the cache
    if (n_prompt < 1 || n_decode < 0 || n_prompt + n_decode > n_ctx || n_prompt > 512) return -5;
    llama_init_backend(false);
    llama_context_params p = llama_context_default_params();
    p.n_ctx = n_ctx;
    p.n_batch = 512;
    p.n_gpu_layers = n_gpu_layers;
    p.seed = 1;
    const auto t0 = clk::now();
    llama_model *m = llama_load_model_from_file(path, p);
    if (!m) return -1;
    llama_context *c = llama_new_context_with_model(m, p);
    if (!c) {
        llama_free_model(m);
        return -2;
    }
    out[0] = std::chrono::duration<double>(clk::now() - t0).count();
    const int nv = llama_n_vocab(c);
    std::vector<llama_token> toks(n_prompt);
    for (int i = 0; i < n_prompt; i++) toks[i] = i == 0 ? 1 : (llama_token)((i * 7919 + 13) % nv);
    int rc = 0;
    double prompt_ms = 0;
    g_prompt_min_ms = 1e300;
    g_prompt_max_ms = 0.0;
    for (int r = 0; r < reps && rc == 0; r++) {
        const auto a = clk::now();
        rc = llama_eval(c, toks.data(), n_prompt, 0, n_threads) ? -3 : 0;
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - a).count();
        prompt_ms += ms;
        g_prompt_min_ms = ms < g_prompt_min_ms ? ms : g_prompt_min_ms;
        g_prompt_max_ms = ms > g_prompt_max_ms ? ms : g_prompt_max_ms;
    }
    out[1] = prompt_ms / (reps > 0 ? reps : 1);
    const auto a = clk::now();
    for (int i = 0; i < n_decode && rc == 0; i++) {
        const llama_token t = (llama_token)((i * 104729 + 7) % nv);
        rc = llama_eval(c, &t, 1, n_prompt + i, n_threads) ? -4 : 0;
    }
    out[2] = n_decode > 0 ? std::chrono::duration<double, std::milli>(clk::now() - a).count() / n_decode : 0.0;
    if (rc == 0) {
        memcpy(last_logits, llama_get_logits(c), sizeof(float) * (size_t)nv);
        rc = nv;
    }
    llama_free(c);
    llama_free_model(m);
    return rc;
}
