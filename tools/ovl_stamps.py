"""Phase stamps of the overlapped decode chain (GGML_HIP_CHAIN_STAMPS=1), LLaMA-7B shapes, data-dependent
wiring as tools/chain_bench.py.  Per task: workgroup phase times (s_memrealtime, 100 MHz) relative to the
first workgroup start of task 0, median / max over the task's workgroups:
  0 start, 1 ring issued, 2 producer flags seen (wave 0), 3 after barrier, 4 x in LDS, 5 rows done,
  6 stores drained (flag store follows).
Usage: GGML_HIP_CHAIN_STAMPS=1 python tools/ovl_stamps.py [layers] [overlap 0/1]"""
import ctypes
import os
import sys

import numpy as np

os.environ.setdefault("GGML_HIP_CHAIN_STAMPS", "1")
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ovl = int(sys.argv[2]) if len(sys.argv) > 2 else 1
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
Y = [gh.DeviceBuffer(M * 4) for M in (K, K, K, K, F, F, K)]
tasks = []
x = x0
for l in range(layers):
    w = W[l]
    tasks.append((w[0:3], [K, K, K], K, x, Y[0:3]))
    tasks.append(([w[3]], [K], K, Y[0], [Y[3]]))
    tasks.append((w[4:6], [F, F], K, Y[3], Y[4:6]))
    tasks.append(([w[6]], [K], F, Y[4], [Y[6]]))
    x = Y[6]
gh.synchronize()
L.ggml_hip_debug_set_chain_overlap.argtypes = [ctypes.c_int]
L.ggml_hip_debug_set_chain_overlap(ovl)
ch = gh.Chain(tasks)
for _ in range(5):
    ch.launch(s)
gh.synchronize()
assert ch.status() == 0
T = len(tasks)
st = np.zeros((T, 256, 8), np.uint64)
grid = (ctypes.c_int * T)()
L.ggml_hip_debug_chain_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
gh.check(L.ggml_hip_debug_chain_stamps(ch.h, st.ctypes.data, grid))
t0 = min(int(st[0, :grid[0], 0].min()), int(st[0, :grid[0], 0].min()))
names = ["qkv", "wo", "w13", "w2"]
print(f"{'task':>8} {'start0':>7} {'startmax':>8} {'issued':>7} {'flag':>7} {'x':>7} {'rows':>7} {'pub_med':>7} "
      f"{'pub_max':>7}  (us from task 0 start; medians over workgroups)")
prev_pub = None
for t in range(T):
    g = grid[t]
    a = (st[t, :g, :].astype(np.int64) - t0) / 100.0
    med = np.median(a, axis=0)
    print(f"{t:>4}{names[t % 4]:>4} {a[:, 0].min():7.2f} {a[:, 0].max():8.2f} {med[1]:7.2f} {med[2]:7.2f} {med[4]:7.2f} "
          f"{med[5]:7.2f} {med[6]:7.2f} {a[:, 6].max():7.2f}")
# per-layer summary over the middle layers
lay = []
for l in range(1, layers - 1):
    t = 4 * l
    a0 = (st[t, :grid[t], 6].astype(np.int64).max() - t0) / 100.0
    a1 = (st[t + 4, :grid[t + 4], 6].astype(np.int64).max() - t0) / 100.0
    lay.append(a1 - a0)
print(f"layer period (publish max to publish max, layers 1..{layers - 2}): median {np.median(lay):.2f} us")
hop = []
for t in range(1, T):
    p = (st[t - 1, :grid[t - 1], 6].astype(np.int64).max() - t0) / 100.0
    f = np.median((st[t, :grid[t], 2].astype(np.int64) - t0) / 100.0)
    xr = np.median((st[t, :grid[t], 4].astype(np.int64) - t0) / 100.0)
    hop.append((f - p, xr - f))
hop = np.array(hop)
print(f"producer published (max) -> consumer flag seen (median): {np.median(hop[:, 0]):.2f} us; flag -> x in LDS: "
      f"{np.median(hop[:, 1]):.2f} us")
