"""The attention's f16 x f32 mul_mat (ggml_compute_forward_mul_mat_f16_f32, ggml.c:11026, with
ggml_vec_dot_f16 ggml.c:2303): the LDS-tiled kernel (prefill, many src1 rows) against the
one-group-per-output kernel, bit for bit, on the strided layouts llama.cpp hands it (the permuted
K cache, the transposed V cache) and on K with and without a tail past the last 32-element step.
The one-group kernel itself is pinned bitwise against the reference's CPU build end to end
(tests/test_gpu_llama_ggjt.py); the numpy restatement below checks both to within an ulp (numpy
has no fused multiply-add, so its chains are formed in float64 and rounded once per step)."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


def ref_dot_f16(x16, y32):
    """ggml_vec_dot_f16, AVX F16 schedule: 32 chains, GGML_F32x8_REDUCE, tail in double."""
    K = x16.shape[0]
    x = x16.astype(np.float64)
    y = y32.astype(np.float16).astype(np.float64)
    np_ = K & ~31
    acc = np.zeros(32, np.float32)
    for s in range(0, np_, 32):
        acc = (acc.astype(np.float64) + x[s:s + 32] * y[s:s + 32]).astype(np.float32)
    a = acc[0:8] + acc[16:24]
    b = acc[8:16] + acc[24:32]
    c = a + b
    t = c[0:4] + c[4:8]
    res = np.float32(np.float32(t[0] + t[1]) + np.float32(t[2] + t[3]))
    s = float(res)
    for e in range(np_, K):
        s += float(np.float32(np.float32(x[e]) * np.float32(y[e])))
    return np.float32(s)


def run(L, src0, src1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12, tiled, merged=None):
    L.ggml_hip_debug_f16_mul_mat.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_int64] * 7 + \
        [ctypes.c_void_p, ctypes.c_int]
    ggml_hip.check(L.ggml_hip_debug_f16_mul_mat(src0.ptr, src1.ptr, d.ptr, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12,
                                                merged.ptr if merged is not None else None, tiled), "f16 mul_mat")


# (name, K, ne01, ne11, ne02, layout): "kq" = src0 rows K f16 values apart by n_embd (the permuted
# K cache), src1 = permuted Q; "kqv" = src0 = the transposed V cache (rows n_ctx apart), src1 = the
# contiguous soft_max output
CASES = [("kq_small", 128, 40, 40, 4, "kq"), ("kqv_tail8", 40, 128, 40, 4, "kqv"),
         ("kq_ragged", 64, 37, 19, 3, "kq"), ("kqv_k1", 1, 64, 9, 2, "kqv"), ("kqv_k31", 31, 64, 17, 2, "kqv"),
         ("kqv_k33", 33, 64, 17, 2, "kqv"), ("kq_500", 128, 500, 500, 2, "kq"), ("kqv_500", 500, 128, 500, 2, "kqv")]


@pytest.mark.parametrize("name,K,ne01,ne11,ne02,layout", CASES, ids=[c[0] for c in CASES])
def test_tiled_matches_grouped_bitwise(name, K, ne01, ne11, ne02, layout):
    L = ggml_hip.load()
    rng = np.random.default_rng(K * 1000 + ne01 + ne11)
    if layout == "kq":           # cache_k [n_ctx][n_embd] f16, head i2 at columns 128*i2: row stride n_embd
        n_embd = K * ne02
        cache = (rng.standard_normal((ne01, n_embd)) * 0.5).astype(np.float16)
        nb01, nb02 = n_embd * 2, K * 2
        q = rng.standard_normal((ne11, ne02, K)).astype(np.float32)   # [token][head][dim]
        src1, nb11, nb12 = q, ne02 * K * 4, K * 4
        x_of = lambda i2, i0: cache[i0, i2 * K:(i2 + 1) * K]
        y_of = lambda i2, i1: q[i1, i2]
    else:                        # cache_v transposed: [head][dim][n_ctx] f16, row stride n_ctx
        n_ctx = K + 7
        cache = (rng.standard_normal((ne02, ne01, n_ctx)) * 0.5).astype(np.float16)
        nb01, nb02 = n_ctx * 2, ne01 * n_ctx * 2
        p = rng.random((ne02, ne11, K)).astype(np.float32)
        p /= p.sum(-1, keepdims=True)
        src1, nb11, nb12 = p, K * 4, ne11 * K * 4
        x_of = lambda i2, i0: cache[i2, i0, :K]
        y_of = lambda i2, i1: p[i2, i1]
    s0, s1 = DB.from_array(cache), DB.from_array(src1)
    nout = ne01 * ne11 * ne02
    outs = []
    for tiled in (0, 1):
        d, m = DB(nout * 4), DB(nout * 4)
        run(L, s0, s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12, tiled, m)
        y = d.download((ne02, ne11, ne01), np.float32)
        merged = m.download((ne11, ne02, ne01), np.float32)
        assert np.array_equal(merged.view(np.uint32), y.transpose(1, 0, 2).view(np.uint32))
        outs.append(y)
    assert np.isfinite(outs[0]).all()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    # spot check against the restatement (within an ulp: numpy has no fma)
    for (i2, i1, i0) in [(0, 0, 0), (ne02 - 1, ne11 - 1, ne01 - 1), (ne02 // 2, ne11 // 2, ne01 // 3)]:
        r = ref_dot_f16(x_of(i2, i0), y_of(i2, i1))
        g = outs[1][i2, i1, i0]
        assert abs(float(g) - float(r)) <= 2 * np.spacing(np.float32(abs(r)) + np.float32(1e-30)), (i2, i1, i0, g, r)


@pytest.mark.parametrize("name,K,ne01,ne11,ne02,layout", CASES, ids=[c[0] for c in CASES])
def test_mfma_fast_mode_within_fp32_bound(name, K, ne01, ne11, ne02, layout):
    """The fast-mode kernel (tiled = 2: v_mfma_f32_32x32x16_f16 on the same fp16 operands; the backend
    takes it for ne11 >= 32 outside exact mode): every output within the fp32-accumulation bound of the
    exact sum of the fp16 products (float64 here), |d - ref| <= 1e-5 * sum|x * fp16(y)| + 1e-30, on the
    strided K / V cache layouts, K tails past the last 16-element step and ragged tiles; merged copy
    bitwise equal to dst."""
    L = ggml_hip.load()
    rng = np.random.default_rng(K * 7 + ne01 * 3 + ne11)
    if layout == "kq":
        n_embd = K * ne02
        cache = (rng.standard_normal((ne01, n_embd)) * 0.5).astype(np.float16)
        nb01, nb02 = n_embd * 2, K * 2
        q = rng.standard_normal((ne11, ne02, K)).astype(np.float32)
        src1, nb11, nb12 = q, ne02 * K * 4, K * 4
        X = np.stack([cache[:, i2 * K:(i2 + 1) * K] for i2 in range(ne02)])        # [i2][i0][K]
        Y = q.transpose(1, 0, 2)                                                   # [i2][i1][K]
    else:
        n_ctx = K + 7
        cache = (rng.standard_normal((ne02, ne01, n_ctx)) * 0.5).astype(np.float16)
        nb01, nb02 = n_ctx * 2, ne01 * n_ctx * 2
        p = rng.random((ne02, ne11, K)).astype(np.float32)
        p /= p.sum(-1, keepdims=True)
        src1, nb11, nb12 = p, K * 4, ne11 * K * 4
        X, Y = cache[:, :, :K], p
    s0, s1 = DB.from_array(cache), DB.from_array(src1)
    nout = ne01 * ne11 * ne02
    d, m = DB(nout * 4), DB(nout * 4)
    run(L, s0, s1, d, K, ne01, ne11, ne02, nb01, nb02, nb11, nb12, 2, m)
    y = d.download((ne02, ne11, ne01), np.float32)
    merged = m.download((ne11, ne02, ne01), np.float32)
    assert np.array_equal(merged.view(np.uint32), y.transpose(1, 0, 2).view(np.uint32))
    x64 = X.astype(np.float64)
    y64 = Y.astype(np.float16).astype(np.float64)
    ref = np.einsum("hik,hjk->hji", x64, y64)
    sab = np.einsum("hik,hjk->hji", np.abs(x64), np.abs(y64))
    err = np.abs(y.astype(np.float64) - ref)
    assert np.isfinite(y).all()
    assert (err <= 1e-5 * sab + 1e-30).all(), float((err / (sab + 1e-30)).max())
