"""A/B of the bench's 4-layer, 512-token prefill (fp6 images, k_gemm9), interleaved rounds, ms per pass:
  indep       each group on a fixed input x (ggml_hip_mul_mat_q4_0_multi; k_prep9_x per group)
  dep_calls   the dependent x pointers (x = the producer's y) through the same separate calls
  chain_prep  ggml_hip_chain_create_n with every image by k_prep9_x (ggml_hip_debug_set_chain_x9(0))
  chain_fold  the same chain, each k_gemm9 epilogue writing the next x image
  python tools/prefill_chain_ab.py [rounds] [modes,comma,separated]
(GGML_HIP_GEMM9_WIDE etc. apply as usual.)"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python"), ROOT]

import ggml_hip as gh  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["indep", "dep_calls", "chain_prep", "chain_fold"]
    import bench
    L = gh.load()
    N, layers, reps = 512, 4, 5
    stream = L.ggml_hip_default_stream()
    stack = bench.Stack(gh, L, 0, 1, layers)
    xs = {}
    for K in (4096, 11008):
        xs[K] = gh.DeviceBuffer(K * 4 * N)
        gh.check(L.ggml_hip_fill_gaussian(xs[K].ptr, K * N, 0x5EED1000 + K, 0.0, 1.0, None))
    for K, M in ((4096, 11008), (11008, 4096)):
        gh.check(L.ggml_hip_reserve_workspace_mm(K, N, M))
    groups = ((0, 1, 2), (3,), (4, 5), (6,))
    ybuf = {i: gh.DeviceBuffer(bench.LAYER[i][2] * 4 * N) for i in range(7)}
    DEP = {0: 6, 3: 0, 4: 3, 6: 4}
    fixed, dep = [], []
    for li, row in enumerate(stack.mats):
        for g in groups:
            K = row[g[0]][1]
            n = len(g)
            wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
            mp = (ctypes.c_int64 * n)(*[row[i][3] for i in g])
            yp = (ctypes.c_void_p * n)(*[ybuf[i].ptr for i in g])
            xd = xs[K].ptr if (li == 0 and g[0] == 0) else ybuf[DEP[g[0]]].ptr
            fixed.append((n, wp, mp, K, xs[K].ptr, yp))
            dep.append((n, wp, mp, K, xd, yp))
    tasks = [([row[i][4].ptr for i in g], [row[i][3] for i in g], row[g[0]][1],
              xs[row[g[0]][1]].ptr if (li == 0 and g[0] == 0) else ybuf[DEP[g[0]]].ptr, [ybuf[i].ptr for i in g])
             for li, row in enumerate(stack.mats) for g in groups]
    for row in stack.mats:
        for _, K, M, m, buf, _ in row:
            gh.check(L.ggml_hip_weight_image_create(buf.ptr, K, m, stream))
    ch = gh.Chain(tasks, N=N)

    def calls(lst):
        def f():
            for n, wp, mp, K, x, yp in lst:
                gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, x, N, yp, stream))
        return f

    def chain(fold):
        def f():
            gh.check(L.ggml_hip_debug_set_chain_x9(1 if fold else 0))
            ch.launch(stream)
        return f
    fns = {"indep": calls(fixed), "dep_calls": calls(dep), "chain_prep": chain(False), "chain_fold": chain(True)}
    res = {m: [] for m in modes}
    for r in range(rounds):
        for m in modes:
            fns[m]()
            gh.synchronize()
            a, b = gh.Event(), gh.Event()
            a.record(stream)
            for _ in range(reps):
                fns[m]()
            b.record(stream)
            b.synchronize() if hasattr(b, "synchronize") else gh.synchronize()
            res[m].append(round(a.elapsed_ms(b) / reps, 4))
        print(f"round {r}: " + ", ".join(f"{m} {res[m][-1]:.4f}" for m in modes), flush=True)
    ops = sum(2 * K * m * N for row in stack.mats for _, K, M, m, _, _ in row)
    print(json.dumps({m: {"ms_per_pass": v, "best_TOPs": round(ops / (min(v) * 1e-3) / 1e12, 1)} for m, v in res.items()}))
    gh.check(L.ggml_hip_debug_set_chain_x9(-1))


if __name__ == "__main__":
    main()
