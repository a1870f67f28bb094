"""Golden logits of the small GPT-NeoX model (tests/gptneox_model.py) from the REFERENCE's own GPT-NeoX
frontend (arch/gptneox/gptneox.cpp) + ggml.c, CPU-only build (oracle/_ref/libgptneox_ref_cpu.so,
oracle/Makefile `ref`).  Run here (needs the reference build): python tests/golden/gen_gptneox_golden.py"""
import ctypes
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import gptneox_model as G  # noqa: E402


def ref_logits(lib_path, model_path, n_threads=4):
    """(last prompt row of logits [n_vocab], decode-step logits [len(G.DECODE)][n_vocab])"""
    lib = ctypes.CDLL(lib_path)
    lib.refgptneox_logits.restype = ctypes.c_int
    lib.refgptneox_logits.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    toks = np.array(G.PROMPT, np.int32)
    dec = np.array(G.DECODE, np.int32)
    out = np.zeros(G.HP["n_vocab"], np.float32)
    dout = np.zeros((len(dec), G.HP["n_vocab"]), np.float32)
    rc = lib.refgptneox_logits(model_path.encode(), toks.ctypes.data, len(toks), dec.ctypes.data, len(dec), n_threads,
                               out.ctypes.data, dout.ctypes.data)
    if rc != G.HP["n_vocab"]:
        raise RuntimeError(f"refgptneox_logits failed: {rc}")
    return out, dout


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        mp = os.path.join(d, "gptneox-small-q4_0.ggjt")
        sha = G.write(mp)
        logits, dlogits = ref_logits(os.path.join(ROOT, "oracle", "_ref", "libgptneox_ref_cpu.so"), mp)
    np.save(os.path.join(HERE, "gptneox_small_logits.npy"), logits)
    np.save(os.path.join(HERE, "gptneox_small_decode_logits.npy"), dlogits)
    json.dump({"model_sha256": sha, "prompt": G.PROMPT, "decode": G.DECODE, "hparams": G.HP,
               "generator": "reference arch/gptneox/gptneox.cpp + ggml.c (CPU, -march=x86-64-v3), gptneox_eval of "
                            "the prompt at n_past 0 (last row of logits), then one gptneox_eval per decode token at "
                            "n_past = 12, 13, 14; 4 threads"},
              open(os.path.join(HERE, "gptneox_small_manifest.json"), "w"), indent=1)
    print("model", sha, "logits", logits.shape, dlogits.shape, float(np.abs(logits).max()), float(np.abs(dlogits).max()),
          float(logits.std()), int(logits.argmax()), [int(r.argmax()) for r in dlogits])
