"""k_gemm9's two tiles (128 x 64 with its half-tile tail, 128 x 128) per launch shape and token count, and what the
automatic choice (wide_pays) takes: LLaMA-7B / 13B and Falcon-7B prefill launches (sibling groups as their total
rows), registered fp6 images, HIP events over 10 calls (x image + GEMM; the image prep is the same for both).
Usage: python tools/g9_tile_sweep.py > out.json"""
import ctypes
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "llama.cpp-q_4_0_amd", "python")]
import ggml_hip as gh  # noqa: E402

L = gh.load()
L.ggml_hip_debug_set_gemm9_wide.argtypes = [ctypes.c_int]
SHAPES = [(4096, 12288), (4096, 4096), (4096, 22016), (11008, 4096),          # LLaMA-7B q|k|v, wo, w1|w3, w2
          (5120, 15360), (5120, 5120), (5120, 27648), (13824, 5120),          # LLaMA-13B
          (4544, 22848), (4544, 4544), (18176, 4544)]                          # Falcon-7B qkv|fc, dense, fc2
NS = [int(v) for v in os.environ.get("NS", "128 256 384 512 768 1024 2048").split()]
NMAX = max(NS)
out = []
s = L.ggml_hip_default_stream()
# COLD=1: the calls cycle over distinct copies of the weight (> 600 MB of images in all), so every call streams its
# image from HBM as a model's layers do (the default reuses one copy: Infinity-Cache hits)
COLD = os.environ.get("COLD", "0") == "1"
for K, M in SHAPES:
    tmp = gh.DeviceBuffer(K * M * 4)
    gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, 11, 0.0, 0.02, None))
    img = ((M + 127) // 128) * 128 * K // 32 * 26
    ncopy = max(2, -(-600 * 2 ** 20 // img)) if COLD else 1
    ws = []
    for _ in range(ncopy):
        wc = gh.DeviceBuffer(18 * K // 32 * M)
        gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, wc.ptr, None))
        gh.check(L.ggml_hip_weight_image_create(wc.ptr, K, M, None))
        ws.append(wc)
    tmp.free()
    w = ws[0]
    x = gh.DeviceBuffer(K * NMAX * 4)
    gh.check(L.ggml_hip_fill_gaussian(x.ptr, K * NMAX, 9, 0.0, 1.0, None))
    y = gh.DeviceBuffer(M * NMAX * 4)
    gh.check(L.ggml_hip_reserve_workspace_mm(K, NMAX, M))
    for N in NS:
        row = {"K": K, "M": M, "N": N}
        for name, mode in (("base", 0), ("wide", 1), ("auto", -1), ("base2", 0), ("wide2", 1)):
            gh.check(L.ggml_hip_debug_set_gemm9_wide(mode))
            for _ in range(2):
                gh.check(L.ggml_hip_mul_mat_q4_0_ex(w.ptr, K, M, x.ptr, N, y.ptr, M, 2, s))
            a, b = gh.Event(), gh.Event()
            a.record(s)
            for i in range(10):
                gh.check(L.ggml_hip_mul_mat_q4_0_ex(ws[i % len(ws)].ptr, K, M, x.ptr, N, y.ptr, M, 2, s))
            b.record(s)
            gh.check(L.ggml_hip_stream_synchronize(s))
            row[name] = round(a.elapsed_ms(b) * 100, 2)          # us per call
        row["base"] = min(row.pop("base2"), row["base"])
        row["wide"] = min(row.pop("wide2"), row["wide"])
        row["auto_took"] = "wide" if abs(row["auto"] - row["wide"]) < abs(row["auto"] - row["base"]) else "base"
        print(json.dumps(row), flush=True)
        out.append(row)
    gh.check(L.ggml_hip_debug_set_gemm9_wide(-1))
    for wc in ws:
        L.ggml_hip_weight_image_free(wc.ptr)
        wc.free()
    for b_ in (x, y):
        b_.free()
