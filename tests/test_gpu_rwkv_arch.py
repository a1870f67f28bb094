"""The reference's RWKV-4 frontend on the MI355X backend (north_star "the arch/{falcon,gptneox,rwkv}
frontends call it unchanged").

arch/rwkv/rwkv.cpp builds one recurrent graph that evaluates ONE token (rwkv.cpp:1420-1660), so every
Q4_0 mul_mat it issues is a decode GEMV (N = 1): receptance / key / value / output per block, the
channel-mix key {512 -> 2048}, receptance and value {2048 -> 512}, and the head.  It never offloads a
tensor; built with ggml.c's GPU hooks and linked against libggml_hip_cuda.so, those mul_mats reach the
backend through ggml_compute_forward with the weights served from the device residency cache after
their first use.  Layer norms, the time-mix products, the frontend's ggml_map_* custom ops (exp, max,
sigmoid, 1 - x) and the state copies stay on ggml's CPU ops.  Exact mode: outputs (softmax
probabilities) bit-identical to the reference's CPU-only build (golden); fast kernels: within the
propagated north-star tolerance."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

import rwkv_model as G
from conftest import ROOT
from hip_env import ggml_hip, gpu_available

GOLD = os.path.join(ROOT, "tests", "golden")
HIP_LIB = os.path.join(ROOT, "oracle", "_ref", "librwkv_ref_hip.so")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so"),
              pytest.mark.skipif(not os.path.exists(HIP_LIB), reason="oracle/_ref/librwkv_ref_hip.so not built")]

OPS = json.load(open(os.path.join(GOLD, "ggml_op_enum.json")))
N_LAYER = G.HP["n_layer"]
N_EVAL = len(G.PROMPT) + len(G.DECODE)            # one eval per token
# Q4_0 mul_mats per eval: 4 time-mix + 3 channel-mix matrices per block, plus the head
MM_PER_EVAL = 7 * N_LAYER + 1
# at the default GGML_HIP_DECODE_MIN_WEIGHTS (2^19 elements) the channel-mix key / value matrices
# (512 x 2048, 2^20) go to the backend; the 512 x 512 matrices and the head stay on ggml's CPU op
MM_DEFAULT = 2 * N_LAYER


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    mp = str(tmp_path_factory.mktemp("rwkv") / "r.ggjt")
    assert G.write(mp) == json.load(open(os.path.join(GOLD, "rwkv_small_manifest.json")))["model_sha256"]
    return mp


def run_rwkv(model, exact, min_weights):
    sys.path.insert(0, GOLD)
    from gen_rwkv_golden import ref_logits
    L = ggml_hip.load()
    L.ggml_hip_debug_set_decode_min_weights.restype = ctypes.c_int64
    L.ggml_hip_debug_set_decode_min_weights.argtypes = [ctypes.c_int64]
    L.ggml_hip_debug_op_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(1 if exact else 0), "set_exact")
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    prev_min = L.ggml_hip_debug_set_decode_min_weights(min_weights)
    n = OPS["GGML_OP_COUNT"]
    c = np.zeros(2 * n + 1 + 9, np.int64)
    ggml_hip.check(L.ggml_hip_debug_op_stats(c.ctypes.data, c.size, 1), "op stats reset")
    try:
        got, dec = ref_logits(HIP_LIB, model)
        ggml_hip.check(L.ggml_hip_debug_op_stats(c.ctypes.data, c.size, 1), "op stats")
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
    finally:
        L.ggml_hip_debug_set_decode_min_weights(prev_min)
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
        L.ggml_hip_set_exact(prev)
    gold = np.load(os.path.join(GOLD, "rwkv_small_logits.npy"))
    dgold = np.load(os.path.join(GOLD, "rwkv_small_decode_logits.npy"))
    return got, dec, gold, dgold, int(c[OPS["GGML_OP_MUL_MAT"]]), (h.value, m.value)


def test_rwkv_frontend_on_backend_exact_mode_bitwise(model):
    """Every Q4_0 mul_mat of the nine one-token evals runs on the MI355X (9 x 85), each weight uploaded
    once and then served from the cache; the outputs are bit for bit the reference CPU build's."""
    got, dec, gold, dgold, n_mm, (hits, misses) = run_rwkv(model, exact=True, min_weights=0)
    assert n_mm == N_EVAL * MM_PER_EVAL, n_mm
    assert misses == MM_PER_EVAL and hits == (N_EVAL - 1) * MM_PER_EVAL, (hits, misses)
    assert np.array_equal(got.view(np.uint32), gold.view(np.uint32))
    assert np.array_equal(dec.view(np.uint32), dgold.view(np.uint32))


def test_rwkv_frontend_on_backend_fast_kernels_default_threshold(model):
    """Default threshold: the channel-mix key / value GEMVs on the backend at every eval.  Fast kernels:
    outputs within the north-star tolerance propagated through 12 blocks and the recurrent state
    (each fast mul_mat is within 1e-3 of the CPU's; the next op re-quantizes to q8_0).  Exact mode
    above is the bitwise check."""
    got, dec, gold, dgold, n_mm, (hits, misses) = run_rwkv(model, exact=False, min_weights=-1)
    assert n_mm == N_EVAL * MM_DEFAULT, n_mm
    assert misses == MM_DEFAULT and hits == (N_EVAL - 1) * MM_DEFAULT
    assert np.isfinite(got).all() and np.isfinite(dec).all()
    scale = max(np.abs(gold).max(), np.abs(dgold).max())
    assert np.abs(got - gold).max() / scale < 3e-2
    assert np.abs(dec - dgold).max() / scale < 3e-2
    assert np.median(np.abs(np.vstack([got[None], dec]) - np.vstack([gold[None], dgold]))) / scale < 5e-3
    rows = np.vstack([got[None], dec]).argmax(1) == np.vstack([gold[None], dgold]).argmax(1)
    assert rows.sum() >= 3, rows
