"""Decode (N=1) GEMV per shape: graph replay over 32 distinct weight matrices (> Infinity Cache),
per-launch us and GB/s, for the LLaMA-7B/13B and Falcon-7B shapes (BASELINE configs 2, 4, 5).
Usage: [ALGO=4] [NTOK=1] python tools/shape_sweep.py [K:M ...]   (ALGO default 1 = fused GEMV)"""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
shapes = [tuple(map(int, a.split(":"))) for a in sys.argv[1:]] or [
    (4096, 4096), (4096, 11008), (11008, 4096), (5120, 5120), (5120, 13824), (13824, 5120),
    (4544, 4672), (4544, 4544), (4544, 18176), (18176, 4544)]
s = L.ggml_hip_default_stream()
ALGO = int(os.environ.get("ALGO", "1"))
NTOK = int(os.environ.get("NTOK", "1"))
NMAT = 32
for K, M in shapes:
    tmp = gh.DeviceBuffer(K * M * 4)
    ws = []
    for i in range(NMAT):
        b = gh.DeviceBuffer(18 * K // 32 * M)
        gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 500 + i, 0.0, 0.02, None))
        gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, b.ptr, None))
        ws.append(b)
    tmp.free()
    x = gh.DeviceBuffer(NTOK * K * 4)
    gh.check(L.ggml_hip_fill_gaussian(x.ptr, NTOK * K, 9, 0.0, 1.0, None))
    y = gh.DeviceBuffer(NTOK * M * 4)

    def run():
        for w in ws:
            gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, NTOK, y.ptr, M, ALGO, s))
    run()
    gh.check(L.ggml_hip_stream_synchronize(s))
    g = gh.Graph(s)
    with g:
        run()
    g.launch()
    gh.check(L.ggml_hip_stream_synchronize(s))
    a, b = gh.Event(), gh.Event()
    a.record(s)
    for _ in range(10):
        g.launch()
    b.record(s)
    t = a.elapsed_ms(b) * 1e-3 / (10 * NMAT)
    nbytes = 18 * K // 32 * M + 4 * K + 4 * M
    npairs = K // 64
    print(json.dumps({"algo": ALGO, "N": NTOK, "K": K, "M": M, "pairs": npairs, "chunk_fill": round(npairs / (64 * -(-npairs // 64)), 3),
                      "us": round(t * 1e6, 2), "GBps": round(nbytes / t / 1e9, 1)}), flush=True)
    del g
    for w in ws:
        w.free()
