"""GGML_HIP_GEMM9_MIXED=1: a launch whose 128 x 128 tiles would leave a last round at most half full runs one round of
128 x 128 tiles (row tiles [0, R)) and the rest as 128 x 64.  Checks that the automatic choice's rows [0, 128 R) are
bitwise the forced 128 x 128 tile's and the rest bitwise the forced 128 x 64 tile's, and times auto against both
(HIP events over 10 calls, us per call incl. the x image prep).  Usage: GGML_HIP_GEMM9_MIXED=0|1 python ..."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
L.ggml_hip_debug_set_gemm9_wide.argtypes = [ctypes.c_int]
mixed = os.environ.get("GGML_HIP_GEMM9_MIXED", "0") == "1"
s = L.ggml_hip_default_stream()
SHAPES = [(4096, 12288, 384), (4096, 12288, 512), (4096, 22016, 256), (5120, 15360, 384), (5120, 5120, 1024),
          (13824, 5120, 1024), (4544, 22848, 256), (4544, 4544, 1024), (18176, 4544, 1024),
          # last 128 x 128 round at most half full after two or more whole rounds
          (4096, 12288, 768), (4544, 4544, 2048), (18176, 4544, 2048), (5120, 5120, 2048), (13824, 5120, 2048),
          (5120, 27648, 512), (4096, 22016, 1024)]
if os.environ.get("SHAPES") == "long":
    SHAPES = SHAPES[9:]
for K, M, N in SHAPES:
    tmp = gh.DeviceBuffer(K * M * 4)
    w = gh.DeviceBuffer(18 * K // 32 * M)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 11, 0.0, 0.02, None))
    gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
    tmp.free()
    gh.check(L.ggml_hip_weight_image_create(w.ptr, K, M, None))
    x = gh.DeviceBuffer(K * N * 4)
    gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * N, 9, 0.0, 1.0, None))
    y = gh.DeviceBuffer(M * N * 4)
    gh.check(L.ggml_hip_reserve_workspace_mm(K, N, M))
    row = {"K": K, "M": M, "N": N, "mixed": mixed}
    out = {}
    for name, mode in (("base", 0), ("wide", 1), ("auto", -1)):
        gh.check(L.ggml_hip_debug_set_gemm9_wide(mode))
        gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, N, y.ptr, M, 2, s))
        gh.check(L.ggml_hip_stream_synchronize(s))
        out[name] = y.download((N, M), np.float32).view(np.uint32).copy()
        best = 1e9
        for _ in range(2):
            a, b = gh.Event(), gh.Event()
            a.record(s)
            for _ in range(10):
                gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, N, y.ptr, M, 2, s))
            b.record(s)
            gh.check(L.ggml_hip_stream_synchronize(s))
            best = min(best, a.elapsed_ms(b) * 100)
        row[name] = round(best, 2)
    gh.check(L.ggml_hip_debug_set_gemm9_wide(-1))
    if mixed:
        Nyw = (N + 127) // 128
        tiles_w = (M + 127) // 128 * Nyw
        R = (tiles_w // 256) * 256 // Nyw
        cut = min(M, 128 * R)
        row["rows_wide"] = cut
        row["bitwise_split"] = bool(np.array_equal(out["auto"][:, :cut], out["wide"][:, :cut]) and
                                    np.array_equal(out["auto"][:, cut:], out["base"][:, cut:]))
    print(json.dumps(row), flush=True)
    L.ggml_hip_weight_image_free(w.ptr)
    for b_ in (w, x, y):
        b_.free()
