"""Tiny GGJT LLaMA through the reference llama.cpp on the backend: logit error vs the golden CPU
logits under one configuration (env set by the caller).  Usage: python tools/llama_diag.py THREADS EVALS"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests", "golden")]
from gen_llama_golden import ref_logits  # noqa: E402
import ggjt_model as G  # noqa: E402

nt, ne = int(sys.argv[1]), int(sys.argv[2])
d = tempfile.mkdtemp()
mp = os.path.join(d, "m.ggjt")
G.write(mp)
got = ref_logits(os.path.join(ROOT, "oracle", "_ref", "libllama_ref_hip.so"), mp, n_threads=nt, n_evals=ne)
gold = np.load(os.path.join(ROOT, "tests", "golden", "llama_tiny_logits.npy"))
scale = np.abs(gold).max()
row = np.abs(got - gold).max(1) / scale
print("CFG", os.environ.get("CFG", ""), "threads", nt, "evals", ne, "err", float(row.max()),
      "rows>1e-4", int((row > 1e-4).sum()), "first_bad", int(np.argmax(row > 1e-4)) if (row > 1e-4).any() else -1,
      "per-row", np.array2string(row[:12], precision=1), flush=True)
