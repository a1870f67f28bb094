"""Where the decode engine's time goes (q4_0_engine.hip): the bench's LLaMA-7B chain (32 layers, 128 tasks,
each task's x = an output of the task before) on the engine, timed with HIP events, in the production mode
and the diagnostic modes (GGML_HIP_ENGINE_DIAG: 1 = the gather takes granules unchecked (no edge waits),
2 = no row arithmetic, 3 = both: the loader alone), then one launch with per-CU stamps
(GGML_HIP_ENGINE_STAMPS=1): per task, over CUs, the time from a CU's task start to x in LDS (edge wait) and
to its last row (compute), the loader's ring-full waits and wave 0's waits for landed lines.

  python tools/engine_stamps.py [layers]
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python"), ROOT]

import ggml_hip as gh  # noqa: E402


def build(L, layers):
    import bench
    stack = bench.Stack(gh, L, 0, 1, layers)
    x0 = gh.DeviceBuffer(4096 * 4)
    gh.check(L.ggml_hip_fill_gaussian(x0.ptr, 4096, 0x5EED1000 + 4096, 0.0, 1.0, None))
    yb = {i: gh.DeviceBuffer(bench.LAYER[i][2] * 4) for i in range(7)}
    groups = [[0, 1, 2], [3], [4, 5], [6]]
    DEP = {0: 6, 3: 0, 4: 3, 6: 4}
    tasks = []
    for li, row in enumerate(stack.mats):
        for g in groups:
            x = x0.ptr if (li == 0 and g[0] == 0) else yb[DEP[g[0]]].ptr
            tasks.append(([row[i][4].ptr for i in g], [row[i][3] for i in g], row[g[0]][1], x, [yb[i].ptr for i in g]))
    return stack, x0, yb, tasks


def time_chain(ch, stream, reps=20):
    ch.launch(stream)
    gh.synchronize()
    g = gh.Graph(stream)
    with g:
        ch.launch(stream)
    for _ in range(3):
        g.launch()
    a, b = gh.Event(), gh.Event()
    a.record(stream)
    for _ in range(reps):
        g.launch()
    b.record(stream)
    ms = a.elapsed_ms(b) / reps
    del g
    return ms


def main():
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    L = gh.load()
    L.ggml_hip_debug_engine_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    L.ggml_hip_debug_engine_stamps.restype = ctypes.c_int
    stream = L.ggml_hip_default_stream()
    stack, x0, yb, tasks = build(L, layers)
    res = {"layers": layers}
    # per-launch reference
    ch = gh.Chain(tasks)
    res["launches_ms"] = round(time_chain(ch, stream), 4)
    del ch
    for diag in [int(v) for v in os.environ.get("ENGINE_DIAGS", "0,1,2,3").split(",")]:
        os.environ["GGML_HIP_ENGINE_DIAG"] = str(diag)
        os.environ["GGML_HIP_ENGINE_STAMPS"] = "0"
        ch = gh.Chain(tasks, engine=1)
        res[f"engine_diag{diag}_ms"] = round(time_chain(ch, stream), 4)
        res[f"engine_diag{diag}_status"] = ch.status()
        del ch
        # the same mode once more with stamps: the loader's ring-full waits and wave 0's waits for landed lines
        os.environ["GGML_HIP_ENGINE_STAMPS"] = "1"
        ch = gh.Chain(tasks, engine=1)
        ch.launch(stream)
        gh.synchronize()
        ncu_ = ch.engine_info()["cus"]
        b = np.zeros(ncu_ * (8 + 6 * 160), np.uint64)
        L.ggml_hip_debug_engine_stamps(ch.h, b.ctypes.data, b.size)
        ch.launch(stream)
        gh.synchronize()
        L.ggml_hip_debug_engine_stamps(ch.h, b.ctypes.data, b.size)
        sd = b.reshape(ncu_, -1).astype(np.int64)
        res[f"engine_diag{diag}_loader_span_ring_wait_landed_wait_us"] = [
            round(float(np.median(sd[:, 1] - sd[:, 0])) / 100, 1), round(float(np.median(sd[:, 2])) / 100, 1),
            round(float(np.median(sd[:, 3])) / 100, 1)]
        del ch
    os.environ["GGML_HIP_ENGINE_DIAG"] = "0"
    os.environ["GGML_HIP_ENGINE_STAMPS"] = "1"
    ch = gh.Chain(tasks, engine=1)
    ch.launch(stream)
    gh.synchronize()
    info = ch.engine_info()
    ncu = info["cus"]
    hdr, nt, W = 8, 160, 6
    per = hdr + W * nt
    buf = np.zeros(ncu * per, np.uint64)
    n = L.ggml_hip_debug_engine_stamps(ch.h, buf.ctypes.data, buf.size)        # clears the first launch's
    ch.launch(stream)
    gh.synchronize()
    n = L.ggml_hip_debug_engine_stamps(ch.h, buf.ctypes.data, buf.size)
    assert n == buf.size, n
    st = buf.reshape(ncu, per).astype(np.int64)
    t0 = st[:, 0].min()
    us = lambda v: v / 100.0      # 100 MHz ticks -> us
    res["loader_span_us"] = [round(us(float(np.median(st[:, 1] - st[:, 0]))), 1), round(us(float((st[:, 1] - st[:, 0]).max())), 1)]
    res["loader_ring_wait_us_median_max"] = [round(us(float(np.median(st[:, 2]))), 1), round(us(float(st[:, 2].max())), 1)]
    res["wave0_landed_wait_us_median_max"] = [round(us(float(np.median(st[:, 3]))), 1), round(us(float(st[:, 3].max())), 1)]
    tk = st[:, hdr:].reshape(ncu, nt, W)
    # per task id: over the CUs that have it (start, x ready, wave 0 last row, publish, first row)
    rows = {}
    for c in range(ncu):
        for k in range(nt):
            s0, s1, s2, tid, pub, fr = tk[c, k]
            if s0 == 0:
                continue
            rows.setdefault(int(tid), []).append((s0 - t0, s1 - t0, s2 - t0, (pub - t0) if pub else -1, (fr - t0) if fr else -1))
    lines = []
    tids = sorted(rows)
    for tid in tids[:12] + tids[-4:]:
        a = np.array(rows[tid], np.float64)
        d = {"task": tid, "cus": len(a), "start_med": round(us(np.median(a[:, 0])), 2),
             "x_ready_med": round(us(np.median(a[:, 1])), 2), "x_ready_max": round(us(a[:, 1].max()), 2),
             "gather_wait_med": round(us(np.median(a[:, 1] - a[:, 0])), 2),
             "rows_med": round(us(np.median(a[:, 2] - a[:, 1])), 2), "end_max": round(us(a[:, 2].max()), 2)}
        pub = a[:, 3][a[:, 3] >= 0]
        if pub.size:
            d["publish_last"] = round(us(pub.max()), 2)
        lines.append(d)
    res["tasks"] = lines
    # the edges: the previous task's last granule publish (max over CUs) -> x in LDS -> first row consumed
    e_seen, e_first = [], []
    for i, tid in enumerate(tids[1:], 1):
        prev = np.array(rows[tids[i - 1]], np.float64)
        pubs = prev[:, 3][prev[:, 3] >= 0]
        if not pubs.size:
            continue
        last_pub = pubs.max()
        cur = np.array(rows[tid], np.float64)
        e_seen.append(np.median(cur[:, 1] - last_pub))
        fr = cur[:, 4][cur[:, 4] >= 0]
        if fr.size:
            e_first.append(np.median(fr - cur[:, 1][cur[:, 4] >= 0]))
    res["edge_last_publish_to_x_in_lds_us_median_over_edges"] = round(us(float(np.median(e_seen))), 2) if e_seen else None
    res["edge_last_publish_to_x_in_lds_us_p90"] = round(us(float(np.percentile(e_seen, 90))), 2) if e_seen else None
    res["edge_x_in_lds_to_first_row_us_median"] = round(us(float(np.median(e_first))), 2) if e_first else None
    ends = [us(np.array(rows[t])[:, 2].max()) for t in tids]
    res["task_end_max_us_first8"] = [round(e, 1) for e in ends[:8]]
    res["per_layer_us_from_task_ends"] = round((ends[-1] - ends[3]) / max(1, (len(ends) - 4) / 4), 2) if len(ends) > 8 else None
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
