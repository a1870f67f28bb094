"""Golden logits of the small RWKV model (tests/rwkv_model.py) from the REFERENCE's own RWKV
frontend (arch/rwkv/rwkv.cpp) + ggml.c, CPU-only build (oracle/_ref/librwkv_ref_cpu.so,
oracle/Makefile `ref`).  Run here (needs the reference build): python tests/golden/gen_rwkv_golden.py"""
import ctypes
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import rwkv_model as G  # noqa: E402


def ref_logits(lib_path, model_path):
    """(last prompt row of logits [n_vocab], decode-step logits [len(G.DECODE)][n_vocab])"""
    lib = ctypes.CDLL(lib_path)
    lib.refrwkv_logits.restype = ctypes.c_int
    lib.refrwkv_logits.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p]
    toks = np.array(G.PROMPT, np.int32)
    dec = np.array(G.DECODE, np.int32)
    out = np.zeros(G.HP["n_vocab"], np.float32)
    dout = np.zeros((len(dec), G.HP["n_vocab"]), np.float32)
    rc = lib.refrwkv_logits(model_path.encode(), toks.ctypes.data, len(toks), dec.ctypes.data, len(dec),
                            out.ctypes.data, dout.ctypes.data)
    if rc != G.HP["n_vocab"]:
        raise RuntimeError(f"refrwkv_logits failed: {rc}")
    return out, dout


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        mp = os.path.join(d, "rwkv-small-q4_0.ggjt")
        sha = G.write(mp)
        logits, dlogits = ref_logits(os.path.join(ROOT, "oracle", "_ref", "librwkv_ref_cpu.so"), mp)
    np.save(os.path.join(HERE, "rwkv_small_logits.npy"), logits)
    np.save(os.path.join(HERE, "rwkv_small_decode_logits.npy"), dlogits)
    json.dump({"model_sha256": sha, "prompt": G.PROMPT, "decode": G.DECODE, "hparams": G.HP,
               "generator": "reference arch/rwkv/rwkv.cpp + ggml.c (CPU, -march=x86-64-v3): one rwkv_eval per "
                            "prompt token (recurrent state), logits after the last one, then one rwkv_eval per "
                            "decode token; the frontend computes its graph with 1 thread"},
              open(os.path.join(HERE, "rwkv_small_manifest.json"), "w"), indent=1)
    print("model", sha, "logits", logits.shape, dlogits.shape, float(np.abs(logits).max()), float(np.abs(dlogits).max()),
          float(logits.std()), int(logits.argmax()), [int(r.argmax()) for r in dlogits])
