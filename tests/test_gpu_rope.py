"""Mode-0 rope (ggml_compute_forward_rope_f32) and rope -> cpy into the K cache (llama.cpp:1226-1232) in the
batched elementwise launch the hook runs behind a q4_0 group, against the rope's own kernels, bit for bit:
the two-pairs-per-thread form (16-byte rows and (cos, sin) rows; the K-cache values in one 8- or 16-byte
store when four share a contiguous target row) and the one-pair form it falls back to (a row start off 16
bytes), a cache view off the packed-store alignment, a target row length that is no multiple of 4, F16
and F32 targets, decode and prefill token counts, a partial rotation (n_dims < ne0).  The rotation
itself against numpy (float64 angles) within 2e-5 of the value scale."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer
I64x4 = ctypes.c_int64 * 4


def rope(L, xptr, dptr, cptr, to_f16, ne0, ne1, ne2, n_past, n_dims, nbx, nbd, ne10, ne11, nb10, nb11, nb12, batched):
    L.ggml_hip_debug_rope.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_int64] * 3 + \
        [ctypes.c_int] * 2 + [ctypes.POINTER(ctypes.c_int64)] * 2 + [ctypes.c_int64] * 5 + [ctypes.c_int]
    ggml_hip.check(L.ggml_hip_debug_rope(xptr, dptr, cptr, to_f16, ne0, ne1, ne2, n_past, n_dims, I64x4(*nbx),
                                         I64x4(*nbd), ne10, ne11, nb10, nb11, nb12, batched), "rope")


# (name, head dim, heads, tokens, n_past, n_dims, x byte offset, cache byte offset, target row length, f16)
CASES = [("prefill_f16", 128, 4, 40, 0, 128, 0, 0, None, 1), ("decode_f16", 128, 4, 1, 37, 128, 0, 0, None, 1),
         ("prefill_f32", 128, 4, 33, 5, 128, 0, 0, None, 0), ("head64", 64, 2, 9, 3, 64, 0, 0, None, 1),
         ("x_off8", 128, 2, 7, 0, 128, 8, 0, None, 1), ("cache_off2", 128, 2, 7, 1, 128, 0, 2, None, 1),
         ("row10", 64, 2, 5, 0, 64, 0, 0, 10, 1), ("partial_rot", 128, 2, 6, 4, 64, 0, 0, None, 1),
         ("no_copy", 128, 3, 12, 2, 128, 0, 0, "none", 0)]


@pytest.mark.parametrize("name,hd,nh,nt,n_past,n_dims,xoff,coff,row,f16", CASES, ids=[c[0] for c in CASES])
def test_batched_rope_equals_own_kernel_bitwise(name, hd, nh, nt, n_past, n_dims, xoff, coff, row, f16):
    L = ggml_hip.load()
    rng = np.random.default_rng(hd * 100 + nh * 10 + nt)
    x = (rng.standard_normal((nt, nh, hd)) * 2).astype(np.float32)
    n = x.size
    xb = DB(x.nbytes + 64)
    xb.upload(np.concatenate([np.zeros(xoff // 4, np.float32), x.ravel()]))
    nbx = [4, hd * 4, hd * nh * 4, hd * nh * nt * 4]
    et, es = (np.float16, 2) if f16 else (np.float32, 4)
    outs = {}
    for batched in (1, 0):
        d = DB(x.nbytes)
        cache = np.full(n + 64, 3.0, et)
        cb = DB.from_array(cache)
        if row == "none":
            cptr, ne10, ne11, nb10, nb11, nb12 = None, 0, 0, 0, 0, 0
        elif row is None:                       # the K cache view: 1-d, n values from n_past * n_embd
            cptr, ne10, ne11, nb10, nb11, nb12 = cb.ptr + coff, n, 1, es, n * es, n * es
        else:                                   # a 2-d target of rows of `row` values
            cptr, ne10, ne11, nb10, nb11, nb12 = cb.ptr + coff, row, n // row, es, row * es, n * es
        rope(L, xb.ptr + xoff, d.ptr, cptr, f16, hd, nh, nt, n_past, n_dims, nbx, nbx, ne10, ne11, nb10, nb11, nb12,
             batched)
        outs[batched] = (d.download(x.shape, np.float32), cb.download(cache.shape, et))
    u = np.uint16 if f16 else np.uint32
    assert np.array_equal(outs[1][0].view(np.uint32), outs[0][0].view(np.uint32))
    assert np.array_equal(outs[1][1].view(u), outs[0][1].view(u))
    y = outs[1][0]
    if row != "none":                           # the copy: the rope output in target order, cast
        flat = outs[1][1].view(u)[coff // es:coff // es + n]
        assert np.array_equal(flat, y.ravel().astype(et).view(u))
    # the rotation (pairs below n_dims) against float64 angles theta = p * 10000^(-2i / n_dims)
    p = (n_past + np.arange(nt))[:, None, None].astype(np.float64)
    i = np.arange(n_dims // 2)[None, None, :]
    th = p * 10000.0 ** (-2.0 * i / n_dims)
    x0, x1 = x[..., 0:n_dims:2].astype(np.float64), x[..., 1:n_dims:2].astype(np.float64)
    r0, r1 = x0 * np.cos(th) - x1 * np.sin(th), x0 * np.sin(th) + x1 * np.cos(th)
    scale = np.abs(x).max()
    assert np.abs(y[..., 0:n_dims:2] - r0).max() <= 2e-5 * scale * max(1, n_past + nt) ** 0.5
    assert np.abs(y[..., 1:n_dims:2] - r1).max() <= 2e-5 * scale * max(1, n_past + nt) ** 0.5
