"""Prefill GEMM (N=512, algo 2) per LLaMA-7B shape: graph replay over 8 distinct weight matrices."""
import json, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402
L = gh.load()
s = L.ggml_hip_default_stream()
N = int(os.environ.get("N", 512))
for K, M in [(4096, 4096), (4096, 11008), (11008, 4096)]:
    tmp = gh.DeviceBuffer(K * M * 4)
    ws = []
    for i in range(8):
        b = gh.DeviceBuffer(18 * K // 32 * M)
        gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 700 + i, 0.0, 0.02, None))
        gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, b.ptr, None))
        ws.append(b)
    tmp.free()
    x = gh.DeviceBuffer(K * N * 4); gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * N, 9, 0.0, 1.0, None))
    y = gh.DeviceBuffer(M * N * 4)
    gh.check(L.ggml_hip_reserve_workspace(K, N))
    def run():
        for w in ws:
            gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, N, y.ptr, M, 2, s))
    run(); gh.check(L.ggml_hip_stream_synchronize(s))
    g = gh.Graph(s)
    with g:
        run()
    g.launch(); gh.check(L.ggml_hip_stream_synchronize(s))
    a, b = gh.Event(), gh.Event()
    a.record(s)
    for _ in range(5):
        g.launch()
    b.record(s)
    t = a.elapsed_ms(b) * 1e-3 / (5 * len(ws))
    print(json.dumps({"K": K, "M": M, "N": N, "us": round(t * 1e6, 1), "TOPs": round(2 * M * K * N / t / 1e12, 1)}), flush=True)
    del g
    for w in ws:
        w.free()
