"""Per-wave phase timing of one decode GEMV (GGML_HIP_GEMV_DIAG=7 build path)."""
import ctypes, os, sys
import numpy as np
os.environ.setdefault("GGML_HIP_GEMV_DIAG", "7")
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh
L = gh.load()
L.ggml_hip_debug_gemv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
K = int(os.environ.get("K", 4096)); M = int(os.environ.get("M", 4096))
nmat = 32
ws = []
tmp = gh.DeviceBuffer(K * M * 4)
for i in range(nmat):
    b = gh.DeviceBuffer(18 * K // 32 * M)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 100 + i, 0.0, 0.02, None))
    gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, b.ptr, None)); ws.append(b)
x = gh.DeviceBuffer(K * 4); gh.check(L.ggml_hip_fill_gaussian(x.ptr, K, 7, 0.0, 1.0, None))
y = gh.DeviceBuffer(M * 4)
gh.synchronize()
for r in range(3):
    for i in range(nmat):
        gh.mul_mat(ws[i], K, M, x, 1, y)
    gh.synchronize()
st = np.zeros(8192 * 8, np.uint64)
gh.check(L.ggml_hip_debug_gemv_stamps(st.ctypes.data_as(ctypes.c_void_p), st.size))
nw = (M + 15) // 16 * 16
s = st.reshape(8192, 8)[:min(nw, M)].astype(np.int64)
t0 = s[:, 0].min()
names = ["start", "issued", "quantized", "barrier", "W landed", "item0 done", "end"]
for j, nm in enumerate(names):
    v = (s[:, j] - t0) * 10 / 1000.0   # 100 MHz -> us
    print(f"{nm:12s} min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f} us")
# by wave role: x-waves (wave index < XW within the workgroup) vs the others
XW = int(os.environ.get("XW", 4))
wave_in_wg = np.arange(s.shape[0]) % 16
for role, sel in (("x-waves", wave_in_wg < XW), ("row-only", wave_in_wg >= XW)):
    for j in (4, 6):
        v = (s[sel, j] - t0) * 10 / 1000.0
        print(f"{role:9s} {names[j]:10s} med {np.median(v):6.2f} p90 {np.percentile(v, 90):6.2f} max {v.max():6.2f} us")
