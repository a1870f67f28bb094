"""The prefill attention's f16 x f32 mul_mats of a 500-token LLaMA-7B prompt (32 heads, head_dim 128):
KQ (K = 128, 500 keys x 500 queries) and KQV (K = 500 keys, 128 dims x 500 queries) through
ggml_hip_debug_f16_mul_mat, tiled = 2 (fast-mode MFMA kernel) or TILED env; time them with rocprofv3.
Usage: [TILED=2] python tools/f16_mm_one.py"""
import ctypes
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
L.ggml_hip_debug_f16_mul_mat.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_int64] * 7 + \
    [ctypes.c_void_p, ctypes.c_int]
tiled = int(os.environ.get("TILED", 2))
H, D, T, NCTX = 32, 128, 500, 512
rng = np.random.default_rng(1)
kc = gh.DeviceBuffer.from_array((rng.standard_normal((NCTX, H * D)) * 0.5).astype(np.float16))   # K cache
vc = gh.DeviceBuffer.from_array((rng.standard_normal((H, D, NCTX)) * 0.5).astype(np.float16))   # V cache^T
q = gh.DeviceBuffer.from_array(rng.standard_normal((T, H, D)).astype(np.float32))
sm = gh.DeviceBuffer.from_array(rng.random((H, T, T)).astype(np.float32))
kq, kqv, merged = gh.DeviceBuffer(H * T * T * 4), gh.DeviceBuffer(H * T * D * 4), gh.DeviceBuffer(H * T * D * 4)
for _ in range(10):
    gh.check(L.ggml_hip_debug_f16_mul_mat(kc.ptr, q.ptr, kq.ptr, D, T, T, H, H * D * 2, D * 2, H * D * 4, D * 4, None,
                                          tiled), "KQ")
    gh.check(L.ggml_hip_debug_f16_mul_mat(vc.ptr, sm.ptr, kqv.ptr, T, D, T, H, NCTX * 2, D * NCTX * 2, T * 4, T * T * 4,
                                          merged.ptr, tiled), "KQV")
print("ok")
