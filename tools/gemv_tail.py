"""Per-wave timing of one decode GEMV launch (diagnostic library built with -DGEMV_STAMPS):
  FILE=q4_0_gemv bash tools/build_variant.sh stamps -DGEMV_STAMPS
  GGML_HIP_LIB=variants/libggml_hip_stamps.so python tools/gemv_tail.py
For each LLaMA-7B decode launch shape, the launch is enqueued right behind another GEMV (as in the
bench's graph) 20 times; per launch every wave's s_memrealtime stamps (start, x in LDS, end; 100 MHz)
give the dispatch ramp, the x prologue and the tail (how long the last waves run past the median)."""
import ctypes
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
L.ggml_hip_debug_gemv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
stream = L.ggml_hip_default_stream()


def mats(K, Ms, seed):
    tmp = gh.DeviceBuffer(K * max(Ms) * 4)
    out = []
    for i, M in enumerate(Ms):
        b = gh.DeviceBuffer(18 * K // 32 * M)
        gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, seed + i, 0.0, 0.02, None))
        gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, b.ptr, None))
        out.append(b)
    return out


SHAPES = {"q|k|v": (4096, [4096, 4096, 4096]), "wo": (4096, [4096]), "w1|w3": (4096, [11008, 11008]),
          "w2": (11008, [4096])}
xs = {K: gh.DeviceBuffer(K * 4) for K in (4096, 11008)}
for K, b in xs.items():
    gh.check(L.ggml_hip_fill_gaussian(b.ptr, K, 3 + K, 0.0, 1.0, None))
ys = [gh.DeviceBuffer(11008 * 4) for _ in range(4)]
W = {name: mats(K, Ms, 100 * i) for i, (name, (K, Ms)) in enumerate(SHAPES.items())}


def launch(name):
    K, Ms = SHAPES[name]
    n = len(Ms)
    wp = (ctypes.c_void_p * n)(*[b.ptr for b in W[name]])
    mp = (ctypes.c_int64 * n)(*Ms)
    yp = (ctypes.c_void_p * n)(*[y.ptr for y in ys[:n]])
    gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xs[K].ptr, 1, yp, stream))


PRED = {"q|k|v": "w2", "wo": "q|k|v", "w1|w3": "wo", "w2": "w1|w3"}      # the launch before it in a layer
st = gh.DeviceBuffer(8192 * 16 * 4 * 8)
for name, (K, Ms) in SHAPES.items():
    M = sum(Ms)
    # wo and w2 share M = 4096: stamps select by M, so the predecessor of each must not have the same M
    gh.check(L.ggml_hip_debug_gemv_stamps(st.ptr, M), "stamps")
    starts, xr, ends, tails, ramps = [], [], [], [], []
    for rep in range(22):
        st_np = np.zeros(8192 * 16 * 4, np.uint64)
        gh.check(L.ggml_hip_memcpy_h2d(st.ptr, st_np.ctypes.data, st_np.nbytes, None), "zero stamps")
        if os.environ.get("NOPRED") != "1":
            launch(PRED[name])
        else:
            gh.check(L.ggml_hip_stream_synchronize(stream))
        launch(name)
        gh.check(L.ggml_hip_stream_synchronize(stream))
        a_all = st.download((8192 * 16, 4), np.uint64)
        wid = np.flatnonzero(a_all[:, 0] != 0)            # global wave id = blockIdx * 16 + wave
        a = a_all[wid]
        if rep < 2 or len(a) == 0:
            continue
        t0 = a[:, 0].min()
        s = (a[:, 0] - t0) / 100.0            # us
        x = (a[:, 1] - t0) / 100.0
        e = (a[:, 2] - t0) / 100.0
        starts.append(np.percentile(s, [50, 100]))
        xr.append(np.percentile(x, [50, 100]))
        ends.append(np.percentile(e, [10, 50, 90, 99, 100]))
        tails.append(e.max() - np.median(e))
    S, X, E = np.mean(starts, 0), np.mean(xr, 0), np.mean(ends, 0)
    print(f"{name:6s} M={M:5d} waves={len(a):5d}: start p50 {S[0]:.2f} max {S[1]:.2f} | x-ready p50 {X[0]:.2f} max "
          f"{X[1]:.2f} | end p10 {E[0]:.2f} p50 {E[1]:.2f} p90 {E[2]:.2f} p99 {E[3]:.2f} max {E[4]:.2f} us "
          f"(tail max-p50 {np.mean(tails):.2f})", flush=True)
    if name in ("q|k|v", "w1|w3"):
        blk = wid // 16
        for lo, hi in ((0, 256), (256, 512)):
            m = (blk >= lo) & (blk < hi)
            if m.any():
                print(f"   blocks [{lo},{hi}): start p50 {np.median(s[m]):.2f} max {s[m].max():.2f}, end p50 "
                      f"{np.median(e[m]):.2f} max {e[m].max():.2f}")
        # start vs block id (deciles of block id)
        q = np.percentile(blk, np.arange(0, 101, 12.5))
        hwv = a[:, 3]
        cuid = ((hwv >> 32) & 0xF) * 4096 + (hwv & 0xFF00)
        same = np.mean([cuid[blk == b][0] == cuid[blk == b + 256][0] for b in range(0, 256, 7) if (blk == b + 256).any()])
        print(f"   block b and b + 256 on the same CU: {same:.2f} of sampled pairs")
        print("   start p50 by block-id octile:", [round(float(np.median(s[(blk >= q[i]) & (blk <= q[i + 1])])), 2)
                                                  for i in range(8)])
    if name == "q|k|v":
        # which waves end last: XCD / CU of the latest 1 %
        hw = a[:, 3]
        xcc = (hw >> 32) & 0xF
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        late = e >= np.percentile(e, 99)
        print("   latest 1 % by XCC:", np.bincount(xcc[late].astype(int), minlength=8).tolist(),
              " by SE:", np.bincount(se[late].astype(int), minlength=8).tolist())
        # per-XCC median end
        print("   per-XCC median end:", [round(float(np.median(e[xcc == i])), 2) for i in range(8)])
        print("   per-XCC median start:", [round(float(np.median(s[xcc == i])), 2) for i in range(8)])
gh.check(L.ggml_hip_debug_gemv_stamps(None, -1))
