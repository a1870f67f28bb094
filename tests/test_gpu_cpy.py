"""ggml_cpy F32 -> F16 / F32 (ggml_compute_forward_dup, ggml.c) on the strided views llama.cpp hands it
(llama.cpp:1233-1245): Vcur = transpose(reshape(V)) stored into the transposed V cache at column n_past,
the copy whose source runs along dim 1 and target along dim 0.  From 64 tokens on, the backend stages it
through 64 x 64 LDS tiles (k_elem_batch kind 2; own node and batched alike); below that, and for every
other layout, one element per thread.  A copy plus one fp16 rounding (round to nearest even, as F16C
and numpy do), so every case is checked bit for bit against numpy, and the cache outside the stored
window keeps its sentinel."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


def cpy(L, xptr, dptr, to_f16, n, ne00, ne01, nb00, nb01, nb02, ne10, ne11, nb10, nb11, nb12, batched):
    L.ggml_hip_debug_cpy_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_int64] * 11 + \
        [ctypes.c_int]
    ggml_hip.check(L.ggml_hip_debug_cpy_f32(xptr, dptr, to_f16, n, ne00, ne01, nb00, nb01, nb02, ne10, ne11, nb10,
                                            nb11, nb12, batched), "cpy")


# (tokens N, n_embd, n_ctx, n_past): decode (N = 1), below / at / past the tile, ragged both ways, 7B's 500
V_CASES = [(1, 128, 16, 5), (63, 130, 80, 3), (64, 64, 64, 0), (65, 96, 200, 7), (300, 512, 512, 0),
           (129, 200, 300, 100), (500, 4096, 512, 0)]


@pytest.mark.parametrize("batched", [0, 1], ids=["node", "batched"])
@pytest.mark.parametrize("to_f16", [1, 0], ids=["f16", "f32"])
@pytest.mark.parametrize("N,n_embd,n_ctx,n_past", V_CASES, ids=[f"N{c[0]}_e{c[1]}" for c in V_CASES])
def test_v_cache_store_bitwise(N, n_embd, n_ctx, n_past, to_f16, batched):
    L = ggml_hip.load()
    rng = np.random.default_rng(N * 131 + n_embd)
    v = (rng.standard_normal((N, n_embd)) * 3).astype(np.float32)   # V = mul_mat(wv, cur): [token][n_embd]
    v[0, 0] = 6.1035156e-05 * 0.75                                     # an fp16 subnormal
    et = np.float16 if to_f16 else np.float32
    es = 2 if to_f16 else 4
    sentinel = np.full((n_embd, n_ctx), 7.0, et)                       # the V cache: [n_embd][n_ctx]
    xs, cs = DB.from_array(v), DB.from_array(sentinel)
    # the view of the cache at column n_past (llama.cpp:1238 ggml_view_2d): an offset pointer
    cpy(L, xs.ptr, cs.ptr + n_past * es, to_f16, N * n_embd, N, n_embd, n_embd * 4, 4, N * n_embd * 4, N, n_embd, es, n_ctx * es,
        n_ctx * n_embd * es, batched)
    got = cs.download((n_embd, n_ctx), et)
    want = sentinel.copy()
    want[:, n_past:n_past + N] = v.T.astype(et)
    u = np.uint16 if to_f16 else np.uint32
    assert np.array_equal(got.view(u), want.view(u))


@pytest.mark.parametrize("batched", [0, 1], ids=["node", "batched"])
def test_contiguous_and_permuted_copies_bitwise(batched):
    """The per-element path keeps every other layout: a contiguous 3-d source into a 1-d F16 view (the K
    cache store) and a permuted source (nb00 > nb01, ne00 < 64) into a contiguous F32 target."""
    L = ggml_hip.load()
    rng = np.random.default_rng(3)
    x = rng.standard_normal((40, 8, 64)).astype(np.float32)          # [token][head][dim]
    xs = DB.from_array(x)
    d = DB(x.size * 2)
    cpy(L, xs.ptr, d.ptr, 1, x.size, 64, 8, 4, 64 * 4, 8 * 64 * 4, x.size, 1, 2, x.size * 2, x.size * 2, batched)
    assert np.array_equal(d.download((x.size,), np.float16).view(np.uint16), x.ravel().astype(np.float16).view(np.uint16))
    y = rng.standard_normal((48, 40)).astype(np.float32)             # transpose(y): ne00 = 48 < 64
    ys = DB.from_array(y)
    d2 = DB(y.size * 4)
    cpy(L, ys.ptr, d2.ptr, 0, y.size, 48, 40, 40 * 4, 4, y.size * 4, 48, 40, 4, 48 * 4, y.size * 4, batched)
    assert np.array_equal(d2.download((40, 48), np.float32).view(np.uint32), y.T.copy().view(np.uint32))
