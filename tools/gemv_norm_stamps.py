"""Per-wave phases of the decode GEMV with and without its norm prologue / epilogue (diagnostic library
built with -DGEMV_STAMPS):
  FILE=q4_0_gemv bash tools/build_variant.sh stamps -DGEMV_STAMPS
  GGML_HIP_LIB=variants/libggml_hip_stamps.so python tools/gemv_norm_stamps.py
Each case runs right behind a wo-shaped GEMV (as in a layer) 22 times; per launch every wave's
s_memrealtime stamps (start, x in LDS, end; 100 MHz): x-ready and end percentiles relative to the first
wave's start."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "llama.cpp-q_4_0_amd", "python"), os.path.join(HERE, "..", "tests")]
import ggml_hip as gh  # noqa: E402
from test_gpu_gemv_epi import GemvEpi, gemv_norm, rand_q4  # noqa: E402

L = gh.load()
L.ggml_hip_debug_gemv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
DB = gh.DeviceBuffer
rng = np.random.default_rng(5)
K, F = 4096, 11008
Wqkv = [DB.from_array(rand_q4(4096, K, rng)) for _ in range(3)]
W13 = [DB.from_array(rand_q4(F, K, rng)) for _ in range(2)]
W2 = [DB.from_array(rand_q4(4096, F, rng))]
Wpred = [DB.from_array(rand_q4(1024, K, rng))]
b = DB.from_array(rng.standard_normal(F).astype(np.float32))
a = DB.from_array(rng.standard_normal(F).astype(np.float32))
w = DB.from_array(np.ones(F, np.float32))
ys = [DB(F * 4) for _ in range(3)]
sc = {k: DB(F * 4).ptr for k in ("sum", "norm", "out")}
cs = DB.from_array(np.ones((64, 2), np.float32))
dk, kc, vc = DB(4096 * 4), DB(4096 * 2 * 64), DB(4096 * 2 * 64)
ep = GemvEpi()
ep.kind[0], ep.d[0], ep.cs[0], ep.ne0[0] = 1, ys[0].ptr, cs.ptr, 128
ep.kind[1], ep.d[1], ep.cs[1], ep.ne0[1] = 1, dk.ptr, cs.ptr, 128
ep.c[1], ep.f16[1], ep.ne10[1], ep.ne11[1], ep.nb10[1], ep.nb11[1], ep.nb12[1] = kc.ptr, 1, 4096, 1, 2, 8192, 8192
ep.kind[2], ep.c[2], ep.f16[2] = 2, vc.ptr, 1
ep.ne10[2], ep.ne11[2], ep.nb10[2], ep.nb11[2], ep.nb12[2] = 1, 4096, 2, 128, 4096 * 128
glu = GemvEpi()
glu.glu = 1
s1, s2 = DB(F * 4), DB(F * 4)
glu.d[0], glu.d[1] = s1.ptr, s2.ptr
CASES = [("qkv plain", Wqkv, [4096] * 3, K, 0, None, None), ("qkv norm", Wqkv, [4096] * 3, K, 1, a, None),
         ("qkv norm+epi", Wqkv, [4096] * 3, K, 1, a, ep), ("w1|w3 plain", W13, [F] * 2, K, 0, None, None),
         ("w1|w3 norm", W13, [F] * 2, K, 1, a, None), ("w1|w3 norm+glu", W13, [F] * 2, K, 1, a, glu),
         ("w2 plain", W2, [4096], F, 0, None, None), ("w2 silu", W2, [4096], F, 2, a, None)]
st = DB(8192 * 16 * 4 * 8)
for name, W, Ms, KK, kind, aa, epi in CASES:
    M = sum(Ms)
    gh.check(L.ggml_hip_debug_gemv_stamps(st.ptr, M), "stamps")
    xr, ends, starts = [], [], []
    for rep in range(22):
        gh.check(L.ggml_hip_memcpy_h2d(st.ptr, np.zeros(8192 * 16 * 4, np.uint64).ctypes.data, 8192 * 16 * 4 * 8, None))
        gemv_norm(L, Wpred, [1024], K, 0, None, b, None, ys[:1])          # the launch before (not stamped)
        gemv_norm(L, W, Ms, KK, kind, aa, b, w if kind == 1 else None, ys[:len(W)], epi=epi, extra=sc)
        A = st.download((8192 * 16, 4), np.uint64)
        A = A[A[:, 0] != 0]
        if rep < 2 or len(A) == 0:
            continue
        t0 = A[:, 0].min()
        starts.append(np.percentile((A[:, 0] - t0) / 100.0, [50, 100]))
        xr.append(np.percentile((A[:, 1] - t0) / 100.0, [50, 100]))
        ends.append(np.percentile((A[:, 2] - t0) / 100.0, [50, 90, 100]))
    S, X, E = np.mean(starts, 0), np.mean(xr, 0), np.mean(ends, 0)
    print(f"{name:16s} M={M:5d}: start p50 {S[0]:.2f} max {S[1]:.2f} | x-ready p50 {X[0]:.2f} max {X[1]:.2f} | "
          f"end p50 {E[0]:.2f} p90 {E[1]:.2f} max {E[2]:.2f} us", flush=True)
gh.check(L.ggml_hip_debug_gemv_stamps(None, -1))
