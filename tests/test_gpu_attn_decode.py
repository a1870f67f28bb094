"""The decode attention in one launch (op_kq_softmax_kqv: KQ of one query row per head computed into LDS, then
scale -> diag_mask_inf -> soft_max -> KQV) against KQ's own launch (k_mul_mat_f16_f32) followed by
op_softmax_kqv, on device pointers through ggml_hip_debug_attn_decode: the softmax rows and the KQV outputs
bitwise equal, on the reference llama.cpp's cache layouts (K rows of n_embd f16 per key, heads hd apart; V
transposed: rows of n_ctx f16), head sizes with and without a 32-element tail, n_kv from 1 to 1,000."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer
P = ctypes.c_void_p
I64 = ctypes.c_int64


def attn(L, fused, kc, q, vc, hd, nh, n_ctx, nkv, reps=0):
    L.ggml_hip_debug_attn_decode.argtypes = [ctypes.c_int, P, I64, I64, P, I64, ctypes.c_int, P, I64, I64, I64, I64, I64,
                                             ctypes.c_int, ctypes.c_float, P, P, P, ctypes.c_int, P]
    n_embd = hd * nh
    kq, sm, kqv = DB(nh * nkv * 4), DB(nh * nkv * 4), DB(nh * hd * 4)
    us = ctypes.c_float(0.0)
    ggml_hip.check(L.ggml_hip_debug_attn_decode(fused, kc.ptr, n_embd * 2, hd * 2, q.ptr, hd * 4, hd, vc.ptr, n_ctx * 2,
                                                hd * n_ctx * 2, nkv, nh, hd, nkv - 1, 1.0 / np.sqrt(hd), kq.ptr, sm.ptr,
                                                kqv.ptr, reps, ctypes.byref(us)), "attn")
    return sm.download((nh, nkv), np.float32), kqv.download((nh, hd), np.float32), us.value


def caches(hd, nh, n_ctx, seed):
    rng = np.random.default_rng(seed)
    n_embd = hd * nh
    kc = DB.from_array((rng.standard_normal((n_ctx, n_embd)) * 0.5).astype(np.float16))
    vc = DB.from_array(rng.standard_normal((n_embd, n_ctx)).astype(np.float16))
    q = DB.from_array(rng.standard_normal(n_embd).astype(np.float32))
    return kc, q, vc


@pytest.mark.parametrize("hd,nh", [(128, 32), (64, 8), (80, 4), (256, 2)])
@pytest.mark.parametrize("nkv", [1, 33, 136, 1000])
def test_fused_decode_attention_bitwise(hd, nh, nkv):
    L = ggml_hip.load()
    n_ctx = 1024
    kc, q, vc = caches(hd, nh, n_ctx, hd + nh + nkv)
    sm1, o1, _ = attn(L, 1, kc, q, vc, hd, nh, n_ctx, nkv)
    sm0, o0, _ = attn(L, 0, kc, q, vc, hd, nh, n_ctx, nkv)
    assert np.isfinite(o1).all()
    assert np.array_equal(sm1.view(np.uint32), sm0.view(np.uint32))
    assert np.array_equal(o1.view(np.uint32), o0.view(np.uint32))
