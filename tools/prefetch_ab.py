"""The bench's LLaMA-7B decode chain (32 layers, 128 launches, each x = an output of the launch before) with and
without the weight prefetcher beside it (ggml_hip_chain_set_prefetch), interleaved rounds, ms per token:
  graph      the chain's launches replayed as one HIP graph (the bench headline's form)
  eager      the same launches issued from the host (the prefetcher's form: it forks a stream beside them)
  pf<D>      eager + the prefetcher D launches ahead
  graph_pf<D> the chain with the prefetcher captured into one graph (fork / join)
Outputs of every form are compared bitwise with the graph's.
  python tools/prefetch_ab.py [rounds] [lookaheads, e.g. 2,4,8]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python"), ROOT, os.path.join(ROOT, "tools")]

import ggml_hip as gh  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    looks = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
    from engine_stamps import build
    L = gh.load()
    stream = L.ggml_hip_default_stream()
    stack, x0, yb, tasks = build(L, 32)
    ch = gh.Chain(tasks)
    reps = 20

    def timed(fn):
        for _ in range(3):
            fn()
        gh.check(L.ggml_hip_stream_synchronize(stream))
        a, b = gh.Event(), gh.Event()
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        gh.check(L.ggml_hip_stream_synchronize(stream))
        return a.elapsed_ms(b) / reps

    def outputs():
        gh.check(L.ggml_hip_stream_synchronize(stream))
        return [yb[i].download((yb[i].nbytes // 4,), np.float32, stream) for i in sorted(yb)]

    g = gh.Graph(stream)
    with g:
        ch.launch(stream)
    g.launch()
    ref = outputs()
    graphs, chs = {}, {}
    for d in looks:                 # one chain per lookahead: a captured graph keeps using its chain's plan
        chs[d] = gh.Chain(tasks)
        chs[d].set_prefetch(d)
        gp = gh.Graph(stream)
        with gp:
            chs[d].launch(stream)
        graphs[d] = gp

    forms = {"graph": lambda: g.launch(), "eager": lambda: ch.launch(stream)}
    res = {k: [] for k in forms}
    for d in looks:
        res[f"pf{d}"] = []
        res[f"graph_pf{d}"] = []
    same = {}
    for r in range(rounds):
        ch.set_prefetch(0)
        for k, fn in forms.items():
            res[k].append(round(timed(fn), 4))
        for d in looks:
            ch.set_prefetch(d)
            res[f"pf{d}"].append(round(timed(lambda: ch.launch(stream)), 4))
            same[f"pf{d}"] = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(outputs(), ref))
            ch.set_prefetch(0)
            res[f"graph_pf{d}"].append(round(timed(graphs[d].launch), 4))
            same[f"graph_pf{d}"] = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(outputs(), ref))
        print(f"round {r}: " + ", ".join(f"{k} {v[-1]:.4f}" for k, v in res.items()), flush=True)
    print(json.dumps({"ms_per_token": res, "bitwise_vs_graph": same, "status": ch.status()}))


if __name__ == "__main__":
    main()
