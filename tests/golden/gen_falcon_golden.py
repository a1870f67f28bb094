"""Golden logits of the small Falcon model (tests/falcon_model.py) from the REFERENCE's own Falcon
frontend (arch/falcon/falcon.cpp) + ggml.c, CPU-only build (oracle/_ref/libfalcon_ref_cpu.so,
oracle/Makefile `ref`).  Run here (needs the reference build): python tests/golden/gen_falcon_golden.py"""
import ctypes
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import falcon_model as F  # noqa: E402


def ref_logits(lib_path, model_path, n_threads=4):
    """(last prompt row of logits [n_vocab], decode-step logits [len(F.DECODE)][n_vocab])"""
    lib = ctypes.CDLL(lib_path)
    lib.reffalcon_logits.restype = ctypes.c_int
    lib.reffalcon_logits.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    toks = np.array(F.PROMPT, np.int32)
    dec = np.array(F.DECODE, np.int32)
    out = np.zeros(F.HP["n_vocab"], np.float32)
    dout = np.zeros((len(dec), F.HP["n_vocab"]), np.float32)
    rc = lib.reffalcon_logits(model_path.encode(), toks.ctypes.data, len(toks), dec.ctypes.data, len(dec), n_threads,
                              out.ctypes.data, dout.ctypes.data)
    if rc != F.HP["n_vocab"]:
        raise RuntimeError(f"reffalcon_logits failed: {rc}")
    return out, dout


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as d:
        mp = os.path.join(d, "falcon-small-q4_0.ggjt")
        sha = F.write(mp)
        logits, dlogits = ref_logits(os.path.join(ROOT, "oracle", "_ref", "libfalcon_ref_cpu.so"), mp)
    np.save(os.path.join(HERE, "falcon_small_logits.npy"), logits)
    np.save(os.path.join(HERE, "falcon_small_decode_logits.npy"), dlogits)
    json.dump({"model_sha256": sha, "prompt": F.PROMPT, "decode": F.DECODE, "hparams": F.HP, "qkv_dim": F.qkv_dim(),
               "generator": "reference arch/falcon/falcon.cpp + ggml.c (CPU, -march=x86-64-v3), falcon_eval of the "
                            "prompt at n_past 0 (last row of logits), then one falcon_eval per decode token at "
                            "n_past = 12, 13, 14; 4 threads"},
              open(os.path.join(HERE, "falcon_small_manifest.json"), "w"), indent=1)
    print("model", sha, "logits", logits.shape, dlogits.shape, float(np.abs(logits).max()), float(np.abs(dlogits).max()))
