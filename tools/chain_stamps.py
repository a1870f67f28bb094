"""Phase stamps of the decode chain kernel (GGML_HIP_CHAIN_STAMPS=1), LLaMA-7B shapes.
Per task: medians over workgroups (us, 100 MHz s_memrealtime) of
  A = compute done (staging full), arr = y published + arrived, poll = all arrivals seen,
  acq = acquire done, xq = next x quantized, c0/c1 = first item start / last row end (slot-0 wave).
Usage: GGML_HIP_CHAIN_STAMPS=1 python tools/chain_stamps.py [layers]"""
import ctypes
import os
import sys

import numpy as np

os.environ.setdefault("GGML_HIP_CHAIN_STAMPS", "1")
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
layers = int(sys.argv[1]) if len(sys.argv) > 1 else 4
K, F = 4096, 11008
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
    tasks += [(w[0:3], [K, K, K], K, x, y[0:3]), ([w[3]], [K], K, y[0], [y[3]]),
              (w[4:6], [F, F], K, y[3], y[4:6]), ([w[6]], [K], F, y[4], [y[6]])]
    x = y[6]
ch = gh.Chain(tasks)
for _ in range(3):
    ch.launch()
gh.synchronize()
T = len(tasks)
grid = ctypes.c_int()
n = 8 * 256 * T
st = np.zeros(n * 2, np.uint64)
L.ggml_hip_debug_chain_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
gh.check(L.ggml_hip_debug_chain_stamps(ch.h, st.ctypes.data, 8 * 256 * T, ctypes.byref(grid)))
G = grid.value
s = st[:8 * G * T].reshape(G, T, 8).astype(np.int64)
t0 = s[:, 0, 5][s[:, 0, 5] > 0].min()
us = (s - t0) / 100.0
names = ["A", "arr", "poll", "acq", "xq", "c0", "c1"]
print(f"grid {G}, tasks {T}; medians over workgroups (us from the first compute start)")
print("task  " + " ".join(f"{n:>8s}" for n in names) + "   A.max arr.max  c1.max  per-task")
prevA = 0.0
for t in range(T):
    row = [np.median(us[:, t, k]) for k in range(7)]
    Amax, c1max, armax = us[:, t, 0].max(), us[:, t, 6].max(), us[:, t, 1].max()
    print(f"{t:4d}  " + " ".join(f"{v:8.2f}" for v in row) + f" {Amax:7.2f} {armax:7.2f} {c1max:7.2f} {row[0] - prevA:8.2f}")
    prevA = row[0]
print("status", ch.status())
