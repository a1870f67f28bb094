"""Does the decode GEMV run faster when its weights are Infinity-Cache (MALL, 256 MiB) resident?  Per launch position
of the bench's LLaMA-7B layer (q|k|v, wo, w1|w3, w2), µs per launch of a graph of 32 launches:
  cold  the 32 layers' weights (each launch streams its own bytes from HBM: the bench's situation)
  warm  32 launches on layer 0's weights (after the first, the bytes are MALL-resident: 9.5-51 MB)
The gap bounds what staging the next launches' weights into the MALL (a prefetcher beside the chain) could win.
  python tools/mall_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python"), ROOT]

import ggml_hip as gh  # noqa: E402


def main():
    import bench
    L = gh.load()
    stream = L.ggml_hip_default_stream()
    stack = bench.Stack(gh, L, 0, 1, 32)
    xs = {}
    for K in (4096, 11008):
        xs[K] = gh.DeviceBuffer(K * 4)
        gh.check(L.ggml_hip_fill_gaussian(xs[K].ptr, K, 0x5EED1000 + K, 0.0, 1.0, None))
    groups = ((0, 1, 2), (3,), (4, 5), (6,))
    yb = {i: gh.DeviceBuffer(bench.LAYER[i][2] * 4) for i in range(7)}
    out = {}
    for g_ in groups:
        def args(li):
            row = stack.mats[li]
            n = len(g_)
            return (n, (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g_]), (ctypes.c_int64 * n)(*[row[i][3] for i in g_]),
                    row[g_[0]][1], (ctypes.c_void_p * n)(*[yb[i].ptr for i in g_]))
        res = {}
        for mode, layers in (("cold", list(range(32))), ("warm", [0] * 32)):
            launches = [args(li) for li in layers]
            g = gh.Graph(stream)
            with g:
                for n, wp, mp, K, yp in launches:
                    gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xs[K].ptr, 1, yp, stream))
            for _ in range(3):
                g.launch()
            gh.check(L.ggml_hip_stream_synchronize(stream))
            e0, e1 = gh.Event(), gh.Event()
            e0.record(stream)
            for _ in range(10):
                g.launch()
            e1.record(stream)
            res[mode] = round(e0.elapsed_ms(e1) * 1e3 / (10 * 32), 3)
            del g
        K = stack.mats[0][g_[0]][1]
        nbytes = sum(bench.q4_bytes(K, stack.mats[0][i][3]) for i in g_)
        res["MB"] = round(nbytes / 1e6, 1)
        res["cold_TBps"] = round(nbytes / res["cold"] / 1e6, 2)
        res["warm_TBps"] = round(nbytes / res["warm"] / 1e6, 2)
        out["+".join(bench.LAYER[i][0] for i in g_)] = res
        print(out, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
