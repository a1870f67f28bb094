"""The reference's unmodified llama.cpp (built with -DGGML_USE_CUBLAS, linked against
libggml_hip_cuda.so) loads the tiny GGJT v3 LLaMA file with its own loader and evaluates a
40-token prompt: ggml.c's can_mul_mat sends every Q4_0 mul_mat of the batch (2 layers x 7 + the
output projection = 15 weight matrices, N = 40) to the MI355X backend, the CPU-backend weights go
through the device residency cache, everything else stays on ggml's CPU ops.  The logits must
match the reference's CPU-only golden logits within the propagated north-star tolerance."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

import ggjt_model as G
from conftest import ROOT
from hip_env import ggml_hip, gpu_available

GOLD = os.path.join(ROOT, "tests", "golden")
HIP_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_hip.so")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so"),
              pytest.mark.skipif(not os.path.exists(HIP_LIB), reason="oracle/_ref/libllama_ref_hip.so not built")]


def run_llama(tmp_path, exact):
    sys.path.insert(0, GOLD)
    from gen_llama_golden import ref_logits
    L = ggml_hip.load()
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(1 if exact else 0), "set_exact")
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    mp = str(tmp_path / "m.ggjt")
    assert G.write(mp) == json.load(open(os.path.join(GOLD, "llama_tiny_manifest.json")))["model_sha256"]
    try:
        got = ref_logits(HIP_LIB, mp, n_evals=2)
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
    finally:
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
        L.ggml_hip_set_exact(prev)
    n_q4 = 7 * G.HP["n_layer"] + 1
    assert (m.value, h.value) == (n_q4, n_q4), "every Q4_0 mul_mat ran on the backend (uploaded once, reused)"
    return got, np.load(os.path.join(GOLD, "llama_tiny_logits.npy"))


def test_reference_llama_on_backend_exact_mode_bitwise(tmp_path):
    got, gold = run_llama(tmp_path, exact=True)
    assert np.array_equal(got.view(np.uint32), gold.view(np.uint32))


def test_reference_llama_on_backend_fast_kernels(tmp_path):
    got, gold = run_llama(tmp_path, exact=False)
    assert np.isfinite(got).all()
    row = np.abs(got - gold).max(1) / np.abs(gold).max()
    assert (row < 1e-5).mean() >= 0.75, row
    assert row.max() < 2e-2, row
    assert (got.argmax(1) == gold.argmax(1)).mean() >= 0.95
