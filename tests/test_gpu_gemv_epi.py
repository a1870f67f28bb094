"""The decode GEMV epilogues at the kernel level (csrc/q4_0_gemv.hip EPI, ghip::GemvEpi), on device pointers
through ggml_hip_debug_gemv_norm:

* EPI 1 (q|k|v behind the attention norm): rope mode 0 of Q in place, rope of K into its own tensor plus
  the F16 copy into a K-cache view, V copied into a transposed V-cache view.  The GEMV outputs are
  bitwise those of the same launch without the epilogue, and the epilogue's values are bitwise the
  unfused ops' (rope as k_elem_batch: x0*cos - x1*sin, x0*sin + x1*cos in float32 without contraction;
  the copy's fp16 rounding to nearest even), checked against numpy float32 on the GEMV's own outputs.
* EPI 2 (w1|w3 behind the ffn norm, interleaved gate / up rows): silu -> mul in the epilogue, bitwise
  ggml_hip's own silu -> mul launch on the same gate / up (ggml's fp16 silu table), blocked (default) and
  strided (GEMV map 0) pairs.
The model-level tests (tests/test_gpu_llama_ggjt.py) pin the whole chain to the reference's logits."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer
P = ctypes.c_void_p


class GemvEpi(ctypes.Structure):          # csrc/q4_0_kernels.h
    _fields_ = [("glu", ctypes.c_int), ("table", P), ("d", P * 4), ("cs", P * 4), ("c", P * 4),
                ("kind", ctypes.c_int * 4), ("f16", ctypes.c_int * 4), ("ne0", ctypes.c_int * 4),
                ("ne10", ctypes.c_int * 4), ("ne11", ctypes.c_int * 4), ("nb10", ctypes.c_int * 4),
                ("nb11", ctypes.c_int * 4), ("nb12", ctypes.c_int * 4)]


def rand_q4(M, K, rng):
    """M rows of valid q4_0 blocks: random nibbles, fp16 scales ~1e-2."""
    nb = K // 32
    blk = np.zeros((M, nb, 18), np.uint8)
    d = (rng.standard_normal((M, nb)) * 0.01).astype(np.float16)
    blk[:, :, 0:2] = d.view(np.uint8).reshape(M, nb, 2)
    blk[:, :, 2:] = rng.integers(0, 256, (M, nb, 16), dtype=np.uint8)
    return blk.reshape(M, nb * 18)


def gemv_norm(L, W, Ms, K, kind, a, b, w, ys, epi=None, reps=0, extra=None):
    L.ggml_hip_debug_gemv_norm.argtypes = [ctypes.c_int, P, P, ctypes.c_int64, ctypes.c_int, P, P, P, P, P, P, P, P,
                                           ctypes.c_int, P]
    n = len(W)
    wp = (P * 4)(*[x.ptr for x in W])
    mp = (ctypes.c_int64 * 4)(*Ms)
    yp = (P * 4)(*[y.ptr for y in ys])
    sc = extra or {}
    us = ctypes.c_float(0.0)
    ggml_hip.check(L.ggml_hip_debug_gemv_norm(n, wp, mp, K, kind, a.ptr if a else None, b.ptr, w.ptr if w else None,
                                              sc.get("sum"), sc.get("norm"), sc.get("out"), yp,
                                              ctypes.byref(epi) if epi is not None else None, reps,
                                              ctypes.byref(us)), "gemv_norm")
    return us.value


def rope_np(x, cs, ne0):
    """k_elem_batch's rope mode 0 on one token: pairs (2j, 2j+1) of each ne0-row with (cos, sin) cs[j]."""
    v = x.reshape(-1, ne0 // 2, 2)
    c, s = cs[:, 0][None, :], cs[:, 1][None, :]
    y = np.empty_like(v)
    y[..., 0] = v[..., 0] * c - v[..., 1] * s
    y[..., 1] = v[..., 0] * s + v[..., 1] * c
    return y.reshape(-1)


@pytest.mark.parametrize("K,hd,nh,vf16", [(4096, 128, 32, True), (4096, 64, 64, False), (5120, 128, 40, True)])
def test_rope_cache_epilogue_bitwise(K, hd, nh, vf16):
    L = ggml_hip.load()
    rng = np.random.default_rng(K + hd + nh)
    M = hd * nh
    W = [DB.from_array(rand_q4(M, K, rng)) for _ in range(3)]
    b = DB.from_array(rng.standard_normal(K).astype(np.float32))
    a = DB.from_array(rng.standard_normal(K).astype(np.float32))
    w = DB.from_array((1.0 + 0.1 * rng.standard_normal(K)).astype(np.float32))
    ref = [DB(M * 4) for _ in range(3)]
    gemv_norm(L, W, [M] * 3, K, 1, a, b, w, ref)
    yq, yk, yv = [r.download((M,), np.float32) for r in ref]
    ang = rng.uniform(-3, 3, hd // 2).astype(np.float32)
    cs = np.stack([np.cos(ang), np.sin(ang)], 1).astype(np.float32)
    csd = DB.from_array(cs)
    n_ctx, pos = 64, 37
    kc = DB.from_array(np.zeros(n_ctx * M, np.float16))             # K cache [n_ctx][M] f16
    vdt = np.float16 if vf16 else np.float32
    vc = DB.from_array(np.zeros(M * n_ctx, vdt))                     # V cache [M][n_ctx] (transposed)
    es = 2 if vf16 else 4
    ys = [DB(M * 4) for _ in range(3)]
    dk = DB(M * 4)
    ep = GemvEpi()
    ep.kind[0], ep.d[0], ep.cs[0], ep.ne0[0] = 1, ys[0].ptr, csd.ptr, hd            # rope Q in place
    ep.kind[1], ep.d[1], ep.cs[1], ep.ne0[1] = 1, dk.ptr, csd.ptr, hd               # rope K -> dk, copy to cache
    ep.c[1], ep.f16[1] = kc.ptr + pos * M * 2, 1
    ep.ne10[1], ep.ne11[1], ep.nb10[1], ep.nb11[1], ep.nb12[1] = M, 1, 2, M * 2, M * 2
    ep.kind[2] = 2                                                                   # V -> transposed cache
    ep.c[2], ep.f16[2] = vc.ptr + pos * es, int(vf16)
    ep.ne10[2], ep.ne11[2], ep.nb10[2], ep.nb11[2], ep.nb12[2] = 1, M, es, n_ctx * es, M * n_ctx * es
    gemv_norm(L, W, [M] * 3, K, 1, a, b, w, ys, epi=ep)
    gq, gk, gv = [y.download((M,), np.float32) for y in ys]
    rq, rk = rope_np(yq, cs, hd), rope_np(yk, cs, hd)
    u32 = lambda x: np.ascontiguousarray(x).view(np.uint32)
    assert np.array_equal(u32(gq), u32(rq))                          # Q roped in place
    assert np.array_equal(u32(gk), u32(yk))                          # K's own output kept
    assert np.array_equal(u32(dk.download((M,), np.float32)), u32(rk))
    assert np.array_equal(u32(gv), u32(yv))
    kcache = kc.download((n_ctx, M), np.float16)
    assert np.array_equal(kcache[pos].view(np.uint16), rk.astype(np.float16).view(np.uint16))
    assert not kcache[:pos].any() and not kcache[pos + 1:].any()
    vcache = vc.download((M, n_ctx), vdt)
    assert np.array_equal(vcache[:, pos], yv.astype(vdt))
    assert not vcache[:, :pos].any() and not vcache[:, pos + 1:].any()


@pytest.mark.parametrize("map_", [-1, 0], ids=["blocked", "strided"])
@pytest.mark.parametrize("K,M", [(4096, 11008), (5120, 13824), (4096, 1000)])
def test_glu_epilogue_bitwise(K, M, map_):
    L = ggml_hip.load()
    rng = np.random.default_rng(K + M)
    W = [DB.from_array(rand_q4(M, K, rng)) for _ in range(2)]
    b = DB.from_array(rng.standard_normal(K).astype(np.float32))
    w = DB.from_array((1.0 + 0.1 * rng.standard_normal(K)).astype(np.float32))
    ref = [DB(M * 4) for _ in range(2)]
    gemv_norm(L, W, [M] * 2, K, 1, None, b, w, ref)
    yg, yu = [r.download((M,), np.float32) for r in ref]
    ys = [DB(M * 4) for _ in range(2)]
    su, pr = DB(M * 4), DB(M * 4)
    ep = GemvEpi()
    ep.glu = 1
    ep.d[0], ep.d[1] = su.ptr, pr.ptr
    L.ggml_hip_debug_set_gemv_policy.argtypes = [ctypes.c_int] * 4
    ggml_hip.check(L.ggml_hip_debug_set_gemv_policy(map_, 0, 1, 0), "policy")
    try:
        gemv_norm(L, W, [M] * 2, K, 1, None, b, w, ys, epi=ep)
    finally:
        L.ggml_hip_debug_set_gemv_policy(-1, 0, 1, 0)
    u32 = lambda x: np.ascontiguousarray(x).view(np.uint32)
    assert np.array_equal(u32(ys[0].download((M,), np.float32)), u32(yg))
    assert np.array_equal(u32(ys[1].download((M,), np.float32)), u32(yu))
    # ggml_hip's own silu -> mul on the same gate / up (k_silu_mul, ggml's fp16 table)
    n_pad = ((M + 63) // 64) * 64
    g2 = np.zeros(n_pad, np.float32)
    u2 = np.zeros(n_pad, np.float32)
    g2[:M], u2[:M] = yg, yu
    ga, ub = DB.from_array(g2), DB.from_array(u2)
    sil, prod, prod_ref = DB(n_pad * 4), DB(n_pad * 4), DB(n_pad * 4)
    nbytes = (n_pad // 32) * 4 * 50
    img, img_ref = DB(nbytes), DB(nbytes)
    L.ggml_hip_debug_x9_producer.argtypes = [ctypes.c_int] + [P] * 7 + [ctypes.c_int64] * 2 + [P] * 2
    ggml_hip.check(L.ggml_hip_debug_x9_producer(2, ga.ptr, ub.ptr, None, None, sil.ptr, prod.ptr, prod_ref.ptr, n_pad, 1,
                                                img.ptr, img_ref.ptr), "silu_mul")
    assert np.array_equal(u32(su.download((M,), np.float32)), u32(sil.download((n_pad,), np.float32)[:M]))
    assert np.array_equal(u32(pr.download((M,), np.float32)), u32(prod_ref.download((n_pad,), np.float32)[:M]))
