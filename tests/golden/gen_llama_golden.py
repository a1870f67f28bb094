"""Golden logits of the tiny GGJT v3 LLaMA (tests/ggjt_model.py) from the REFERENCE's own
llama.cpp + ggml.c, CPU-only build (oracle/_ref/libllama_ref_cpu.so, oracle/Makefile `ref`).
Run here (needs the reference build): python tests/golden/gen_llama_golden.py"""
import ctypes
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import ggjt_model as G  # noqa: E402


def ref_logits(lib_path, model_path, n_threads=4, n_evals=1, n_gpu_layers=0, with_decode=False):
    """Prompt logits [40][n_vocab]; with_decode: also the logits of the G.DECODE single-token steps."""
    lib = ctypes.CDLL(lib_path)
    lib.refllama_logits.restype = ctypes.c_int
    lib.refllama_logits.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_void_p]
    toks = np.array(G.PROMPT, np.int32)
    out = np.zeros((len(toks), G.HP["n_vocab"]), np.float32)
    dec = np.array(G.DECODE if with_decode else [0], np.int32)
    dout = np.zeros((len(dec), G.HP["n_vocab"]), np.float32)
    rc = lib.refllama_logits(model_path.encode(), toks.ctypes.data, len(toks), n_threads, 1, out.ctypes.data, out.size,
                             n_evals, n_gpu_layers, dec.ctypes.data, len(G.DECODE) if with_decode else 0,
                             dout.ctypes.data)
    if rc != G.HP["n_vocab"]:
        raise RuntimeError(f"refllama_logits failed: {rc}")
    return (out, dout) if with_decode else out


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        mp = os.path.join(d, "tiny-q4_0.ggjt")
        sha = G.write(mp)
        logits, dlogits = ref_logits(os.path.join(ROOT, "oracle", "_ref", "libllama_ref_cpu.so"), mp,
                                     with_decode=True)
    np.save(os.path.join(HERE, "llama_tiny_logits.npy"), logits)
    np.save(os.path.join(HERE, "llama_tiny_decode_logits.npy"), dlogits)
    json.dump({"model_sha256": sha, "prompt": G.PROMPT, "decode": G.DECODE, "hparams": G.HP, "n_ff": G.n_ff(),
               "logits_shape": list(logits.shape), "decode_logits_shape": list(dlogits.shape),
               "generator": "reference llama.cpp + ggml.c (CPU, -march=x86-64-v3), llama_eval logits_all, 4 threads; "
                            "then one llama_eval per decode token at n_past = 40, 41, 42"},
              open(os.path.join(HERE, "llama_tiny_manifest.json"), "w"), indent=1)
    print("model", sha, "logits", logits.shape, float(np.abs(logits).max()))
