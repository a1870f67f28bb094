"""Per-wave cycle split of the prefill GEMM (GGML_HIP_GEMM_DIAG=5): compute / staging / barrier."""
import ctypes, os, sys
import numpy as np
os.environ.setdefault("GGML_HIP_GEMM_DIAG", "5")
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh
L = gh.load()
L.ggml_hip_debug_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
K = int(os.environ.get("K", 4096)); M = int(os.environ.get("M", 4096)); N = int(os.environ.get("N", 512))
tmp = gh.DeviceBuffer(K * M * 4)
w = gh.DeviceBuffer(18 * K // 32 * M)
gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 5, 0.0, 0.02, None))
gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
x = gh.DeviceBuffer(K * N * 4); gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * N, 7, 0.0, 1.0, None))
y = gh.DeviceBuffer(M * N * 4)
for r in range(3):
    gh.mul_mat(w, K, M, x, N, y, algo=2)
gh.synchronize()
a, b = gh.Event(), gh.Event()
a.record()
for r in range(10):
    gh.mul_mat(w, K, M, x, N, y, algo=2)
b.record()
print(f"K={K} M={M} N={N}: {a.elapsed_ms(b) / 10 * 1e3:.1f} us per mul_mat (incl. q8_0 quantize)")
nw = (M + 63) // 64 * ((N + 127) // 128) * 8
st = np.zeros(16384 * 4, np.uint64)
gh.check(L.ggml_hip_debug_gemm_stamps(st.ctypes.data_as(ctypes.c_void_p), st.size))
s = st.reshape(16384, 4)[:nw].astype(np.float64)
for j, nm in enumerate(["total", "compute", "staging", "barrier"]):
    print(f"{nm:8s} median {np.median(s[:, j]):9.0f} cycles  ({np.median(s[:, j] / s[:, 0]) * 100:5.1f} % of total)")
