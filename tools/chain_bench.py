"""Decode chain (overlapped launches, two streams) vs the same chain on one stream vs one launch per
mul_mat (graph), LLaMA-7B shapes, data-dependent wiring (wo reads q, w1|w3 read wo's y, w2 reads w1's
y, the next layer reads w2's y).
Usage: python tools/chain_bench.py [layers] [reps]"""
import json
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
K, F = 4096, 11008
s = L.ggml_hip_default_stream()
tmp = gh.DeviceBuffer(K * F * 4)


def wq(Kk, M, seed):
    b = gh.DeviceBuffer(18 * Kk // 32 * M)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, Kk * M, seed, 0.0, 0.02, None))
    gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, Kk, M, b.ptr, None))
    return b


W = [[wq(K, K, 16 * l + 0), wq(K, K, 16 * l + 1), wq(K, K, 16 * l + 2), wq(K, K, 16 * l + 3),
      wq(K, F, 16 * l + 4), wq(K, F, 16 * l + 5), wq(F, K, 16 * l + 6)] for l in range(layers)]
x0 = gh.DeviceBuffer(K * 4)
gh.check(L.ggml_hip_fill_gaussian(x0.ptr, K, 1, 0.0, 1.0, None))
Y = [[gh.DeviceBuffer(M * 4) for M in (K, K, K, K, F, F, K)] for _ in range(layers)]
tasks = []
x = x0
for l in range(layers):
    w, y = W[l], Y[l]
    tasks.append((w[0:3], [K, K, K], K, x, y[0:3]))
    tasks.append(([w[3]], [K], K, y[0], [y[3]]))
    tasks.append((w[4:6], [F, F], K, y[3], y[4:6]))
    tasks.append(([w[6]], [K], F, y[4], [y[6]]))
    x = y[6]
gh.synchronize()
nbytes = sum(18 * Kk // 32 * sum(Ms) for _, Ms, Kk, _, _ in tasks)

import ctypes  # noqa: E402
import numpy as np  # noqa: E402

L.ggml_hip_debug_set_chain_overlap.argtypes = [ctypes.c_int]
L.ggml_hip_debug_chain_overlap.argtypes = [ctypes.c_void_p]
ev = [gh.Event(), gh.Event()]


def timeit(fn):
    fn(); gh.synchronize()
    ev[0].record(s)
    for _ in range(reps):
        fn()
    ev[1].record(s)
    return ev[0].elapsed_ms(ev[1]) / reps


def launches():
    for ws, Ms, Kk, xx, ys in tasks:
        gh.mul_mat_multi(ws, Ms, Kk, xx, 1, ys, stream=s)


g = gh.Graph(s)
launches(); gh.synchronize()
with g:
    launches()
ms_g = timeit(g.launch)
yg = Y[-1][6].download((K,), "float32")
out = {"layers": layers, "graph_launches_ms": round(ms_g, 4), "tok_s_launches": round(32 / layers * 1e3 / ms_g, 1)}
for ov in (1, 0):
    L.ggml_hip_debug_set_chain_overlap(ov)
    ch = gh.Chain(tasks)
    tag = "ovl" if ov else "one_stream"
    out[f"{tag}_active"] = L.ggml_hip_debug_chain_overlap(ch.h)
    ms_ce = timeit(lambda: ch.launch(s))
    st_e = ch.status()
    ye = Y[-1][6].download((K,), "float32")
    gc = gh.Graph(s)
    with gc:
        ch.launch(s)
    ms_c = timeit(gc.launch)
    st = ch.status()
    yc = Y[-1][6].download((K,), "float32")
    out.update({f"{tag}_eager_ms": round(ms_ce, 4), f"{tag}_graph_ms": round(ms_c, 4),
                f"{tag}_tok_s_eager": round(32 / layers * 1e3 / ms_ce, 1),
                f"{tag}_tok_s_graph": round(32 / layers * 1e3 / ms_c, 1),
                f"{tag}_GBps_best": round(nbytes / min(ms_c, ms_ce) / 1e6, 1), f"{tag}_status": [st_e, st],
                f"{tag}_bitwise_equal": [bool(np.array_equal(yg.view(np.uint32), ye.view(np.uint32))),
                                         bool(np.array_equal(yg.view(np.uint32), yc.view(np.uint32)))]})
    del gc, ch
L.ggml_hip_debug_set_chain_overlap(-1)
print(json.dumps(out), flush=True)
