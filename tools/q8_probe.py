"""Why does the N = 1 q8_0 quantize launch of exact mode take ~4.8 us (rocprof) for a 16 KB row?
Graph-replays 64 exact mul_mats (algo 4) at K = 4096, N = 1, with M = 16 (one tiny exact workgroup)
and M = 4096, and prints the per-call time; run under rocprofv3 --kernel-trace --stats to split the
quantize and exact kernels."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh
L = gh.load()
s = L.ggml_hip_default_stream()
K = 4096
for M in (16, 4096):
    tmp = gh.DeviceBuffer(K * M * 4)
    w = gh.DeviceBuffer(18 * K // 32 * M)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 3, 0.0, 0.02, None))
    gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
    x = gh.DeviceBuffer(K * 4); gh.check(L.ggml_hip_fill_gaussian(x.ptr, K, 9, 0.0, 1.0, None))
    y = gh.DeviceBuffer(M * 4)
    def run():
        for _ in range(64):
            gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, 1, y.ptr, M, 4, s))
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
    print(f"M={M}: {a.elapsed_ms(b) * 1e3 / (5 * 64):.2f} us per exact mul_mat (quantize + exact)", flush=True)
    del g
