"""Decode attention launch time (LLaMA-7B: 32 heads of 128), one fused launch vs KQ + soft_max/KQV, by n_kv.
usage: attn_ab.py [reps]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "llama.cpp-q_4_0_amd", "python"), os.path.join(HERE, "..", "tests")]
import ggml_hip  # noqa: E402
from test_gpu_attn_decode import attn, caches  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L = ggml_hip.load()
kc, q, vc = caches(128, 32, 2048, 1)
for nkv in (40, 72, 136, 256, 512, 1024, 2048):
    t = {f: attn(L, f, kc, q, vc, 128, 32, 2048, nkv, reps)[2] for f in (1, 0)}
    print(f"n_kv {nkv:5d}: fused {t[1]:7.2f} us   KQ + softmax_kqv {t[0]:7.2f} us", flush=True)
