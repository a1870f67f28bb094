"""Decode GEMV launch times with and without the x prologues and epilogues (LLaMA-7B shapes), through
ggml_hip_debug_gemv_norm: each case launched `reps` times between two HIP events on the backend stream
(consecutive launches: the next one's weights stream while the previous drains, as in a decode).
usage: gemv_epi_ab.py [reps] [rounds]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llama.cpp-q_4_0_amd", "python"))
import ggml_hip  # noqa: E402
from test_gpu_gemv_epi import GemvEpi, gemv_norm, rand_q4  # noqa: E402

DB = ggml_hip.DeviceBuffer


def main(reps=200, rounds=3):
    L = ggml_hip.load()
    rng = np.random.default_rng(7)
    K, M, F = 4096, 4096, 11008
    Wqkv = [DB.from_array(rand_q4(M, K, rng)) for _ in range(3)]
    W13 = [DB.from_array(rand_q4(F, K, rng)) for _ in range(2)]
    W2 = [DB.from_array(rand_q4(M, F, rng))]
    Wo = [DB.from_array(rand_q4(M, K, rng))]
    b = DB.from_array(rng.standard_normal(F).astype(np.float32))
    a = DB.from_array(rng.standard_normal(F).astype(np.float32))
    w = DB.from_array(np.ones(F, np.float32))
    sc = {k: DB(F * 4).ptr for k in ("sum", "norm", "out")}
    yq = [DB(F * 4) for _ in range(3)]
    cs = DB.from_array(np.ones((64, 2), np.float32))
    kc, vc, dk = DB(M * 2 * 64), DB(M * 2 * 64), DB(M * 4)
    ep = GemvEpi()
    ep.kind[0], ep.d[0], ep.cs[0], ep.ne0[0] = 1, yq[0].ptr, cs.ptr, 128
    ep.kind[1], ep.d[1], ep.cs[1], ep.ne0[1] = 1, dk.ptr, cs.ptr, 128
    ep.c[1], ep.f16[1], ep.ne10[1], ep.ne11[1], ep.nb10[1], ep.nb11[1], ep.nb12[1] = kc.ptr, 1, M, 1, 2, M * 2, M * 2
    ep.kind[2], ep.c[2], ep.f16[2] = 2, vc.ptr, 1
    ep.ne10[2], ep.ne11[2], ep.nb10[2], ep.nb11[2], ep.nb12[2] = 1, M, 2, 128, M * 128
    glu = GemvEpi()
    glu.glu = 1
    s1, s2 = DB(F * 4), DB(F * 4)
    glu.d[0], glu.d[1] = s1.ptr, s2.ptr
    L.ggml_hip_debug_set_gemv_policy.argtypes = [ctypes.c_int] * 4
    cases = [
        ("qkv plain", Wqkv, [M] * 3, K, 0, None, None, -1),
        ("qkv norm", Wqkv, [M] * 3, K, 1, a, None, -1),
        ("qkv norm+rope/cache epi", Wqkv, [M] * 3, K, 1, a, ep, -1),
        ("wo plain", Wo, [M], K, 0, None, None, -1),
        ("w1|w3 plain", W13, [F] * 2, K, 0, None, None, -1),
        ("w1|w3 norm", W13, [F] * 2, K, 1, a, None, -1),
        ("w1|w3 norm+glu blocked", W13, [F] * 2, K, 1, a, glu, -1),
        ("w1|w3 norm+glu strided", W13, [F] * 2, K, 1, a, glu, 0),
        ("w2 plain", W2, [M], F, 0, None, None, -1),
        ("w2 silu prologue", W2, [M], F, 2, a, None, -1),
    ]
    res = {c[0]: [] for c in cases}
    for r in range(rounds):
        for name, W, Ms, KK, kind, aa, epi, mp in cases:
            ggml_hip.check(L.ggml_hip_debug_set_gemv_policy(mp, 0, 1, 0))
            us = gemv_norm(L, W, Ms, KK, kind, aa, b, w if kind == 1 else None, yq[:len(W)], epi=epi, reps=reps,
                           extra=sc)
            res[name].append(round(us, 3))
    ggml_hip.check(L.ggml_hip_debug_set_gemv_policy(-1, 0, 1, 0))
    for k, v in res.items():
        print(f"{k:28s} " + " ".join(f"{x:7.3f}" for x in v) + " us")
    print(json.dumps(res))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]])
