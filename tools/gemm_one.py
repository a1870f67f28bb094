"""One prefill GEMM shape timed on the device (the PMC passes of tools/run.sh PARTS=gpmc profile it):
K x M weights (fp6 image built per call under GGML_HIP_GEMM_V=11, or registered once with IMAGE=1), N tokens.
Usage: [K=4096 M=4096 N=512 IMAGE=1] python tools/gemm_one.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
K = int(os.environ.get("K", 4096)); M = int(os.environ.get("M", 4096)); N = int(os.environ.get("N", 512))
tmp = gh.DeviceBuffer(K * M * 4)
w = gh.DeviceBuffer(18 * K // 32 * M)
gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 5, 0.0, 0.02, None))
gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
tmp.free()
if os.environ.get("IMAGE", "1") == "1":
    gh.check(L.ggml_hip_weight_image_create(w.ptr, K, M, None), "image")
x = gh.DeviceBuffer(K * N * 4)
gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * N, 7, 0.0, 1.0, None))
y = gh.DeviceBuffer(M * N * 4)
gh.check(L.ggml_hip_reserve_workspace_mm(K, N, M))
for _ in range(3):
    gh.mul_mat(w, K, M, x, N, y)
gh.synchronize()
a, b = gh.Event(), gh.Event()
a.record()
for _ in range(10):
    gh.mul_mat(w, K, M, x, N, y)
b.record()
us = a.elapsed_ms(b) / 10 * 1e3
print(f"K={K} M={M} N={N}: {us:.1f} us per mul_mat (x image + GEMM), {2 * K * M * N / us / 1e6:.0f} TOP/s")
