"""Split-K MFMA GEMM (algo 3, q4_0 in place) vs the image GEMM (algo 2: k_gemm9 on registered fp6 images)
per token count around the switch (graph replay over 32 distinct weight matrices).
Usage: python tools/n_sweep9.py [K M]"""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
M = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
NMAT = 32
tmp = gh.DeviceBuffer(K * M * 4)
ws = []
for i in range(NMAT):
    b = gh.DeviceBuffer(18 * K // 32 * M)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 300 + i, 0.0, 0.02, None))
    gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, b.ptr, None))
    gh.check(L.ggml_hip_weight_image_create(b.ptr, K, M, None))
    ws.append(b)
tmp.free()
NMAX = 512
x = gh.DeviceBuffer(K * NMAX * 4)
gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * NMAX, 9, 0.0, 1.0, None))
y = gh.DeviceBuffer(M * NMAX * 4)
gh.check(L.ggml_hip_reserve_workspace_mm(K, NMAX, M))
s = L.ggml_hip_default_stream()
for N in [int(v) for v in os.environ.get("NS", "64 96 128 160 192 224 256 320 384 448 512").split()]:
    for algo in (2, 3):
        def run():
            for w in ws:
                gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, N, y.ptr, M, algo, s))
        run()
        gh.check(L.ggml_hip_stream_synchronize(s))
        g = gh.Graph(s)
        with g:
            run()
        g.launch()
        gh.check(L.ggml_hip_stream_synchronize(s))
        a, b = gh.Event(), gh.Event()
        reps = 10
        a.record(s)
        for _ in range(reps):
            g.launch()
        b.record(s)
        t = a.elapsed_ms(b) * 1e-3 / (reps * NMAT)
        print(json.dumps({"K": K, "M": M, "N": N, "path": {2: "gemm9_image", 3: "gemm_sk"}[algo],
                          "us": round(t * 1e6, 2), "TOPs": round(2 * M * K * N / t / 1e12, 1)}), flush=True)
